set -u
cd $GRAFT_REPO_ROOT
b() { env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
for v in "TDE_X=0" "TDE_SPLIT_MINKT=8" "TDE_HWG_MIN_ITEMS=1000" "TDE_SKINNY_M=64" "TDE_SPLIT_MINKT=8 TDE_SKINNY_M=64"; do echo "$v $(b $v)"; done
done
