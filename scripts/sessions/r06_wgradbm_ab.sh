# Round 6: GEMM planner knobs after the 3-waves allocation -- 64-row filter-gradient tiles (TDE_WGRAD_BM64_MAXM), bench alternating.
# Usage: r06_tile_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06zj}
n=0
for v in "base:" "w64a:TDE_WGRAD_BM64_MAXM=100000" "w64s:TDE_WGRAD_BM64_MAXM=1200" "base:" "w64a:TDE_WGRAD_BM64_MAXM=100000" "w64s:TDE_WGRAD_BM64_MAXM=1200"; do
  n=$((n+1)); name=${v%%:*}; vars=${v#*:}
  env $vars timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/bench_${tag}_${name}_$n.json 2> gpurun_out/bench_${tag}_${name}_$n.err || { tail -20 gpurun_out/bench_${tag}_${name}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_${name}_$n.json "$name"
done
