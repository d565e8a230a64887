set -u
cd $GRAFT_REPO_ROOT
for v in "TDE_SPLIT_TARGET=512" "TDE_SPLIT_TARGET=768" "TDE_SPLIT_TARGET=384" "TDE_SPLIT_TARGET=512 TDE_SPLIT_MINKT=8"; do echo "$v"; env $v timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])" || exit 1; done
