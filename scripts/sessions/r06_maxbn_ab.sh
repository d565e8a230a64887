# Round 6: GEMM planner knobs after the 3-waves allocation -- N-tile cap (TDE_MAXBN) per mode, bench alternating.
# Usage: r06_tile_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06zb}
n=0
for v in "base:" "bn64all:TDE_MAXBN=64" "bn64w:TDE_MAXBN=64 TDE_MAXBN_MODES=4" "bn64fd:TDE_MAXBN=64 TDE_MAXBN_MODES=3" "base:" "bn64all:TDE_MAXBN=64" "bn64w:TDE_MAXBN=64 TDE_MAXBN_MODES=4" "bn64fd:TDE_MAXBN=64 TDE_MAXBN_MODES=3"; do
  n=$((n+1)); name=${v%%:*}; vars=${v#*:}
  env $vars timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/bench_${tag}_${name}_$n.json 2> gpurun_out/bench_${tag}_${name}_$n.err || { tail -20 gpurun_out/bench_${tag}_${name}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_${name}_$n.json "$name"
done
