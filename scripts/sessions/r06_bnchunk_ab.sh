# Round 6: GEMM planner knobs after the 3-waves allocation -- BatchNorm partial-sum chunking (TDE_BN_ELEMS, TDE_BN_MAXCH), bench alternating.
# Usage: r06_tile_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06zd}
n=0
for v in "ch512:TDE_BN_MAXCH=512" "ch256:TDE_BN_MAXCH=256" "ch384:TDE_BN_MAXCH=384" "base:" "ch512:TDE_BN_MAXCH=512" "ch256:TDE_BN_MAXCH=256" "ch384:TDE_BN_MAXCH=384" "base:"; do
  n=$((n+1)); name=${v%%:*}; vars=${v#*:}
  env $vars timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/bench_${tag}_${name}_$n.json 2> gpurun_out/bench_${tag}_${name}_$n.err || { tail -20 gpurun_out/bench_${tag}_${name}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_${name}_$n.json "$name"
done
