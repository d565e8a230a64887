#!/bin/bash
# HBM traffic of one bench workload from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE), eager
# mode (the same kernels as the captured graph, one dispatch each), then the per-family summary.
#   bash scripts/pmc.sh TAG [WORKLOAD] [fp32|bf16x3] [BATCH] [extra bench args]
# MATH: fp32|bf16x3|bf16x6|bf16x6r (bench.py --math)
# -> gpurun_out/pmc_<WORKLOAD>_<MATH>_b<BATCH>.json (copy to profiles/ for bench.py's roofline.traffic)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=${1:-r01}
WL=${2:-config2}
MATH=${3:-bf16x6r}
B=${4:-$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(bench.WORKLOADS['$WL'][2])")}
shift $(( $# < 4 ? $# : 4 ))
STEPS=6; WARM=2
# bench.py --no-graph runs 2 eager steps before the timed loop (plain + instrumented)
TOTAL=$((STEPS + WARM + 2))
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc "$C" --kernel-trace -d "$PWD/gpurun_out/pmc_${TAG}_${WL}_$C" -o run \
    --output-format csv -- python3 bench.py --workload "$WL" --steps $STEPS --warmup $WARM --no-graph \
    --no-cpu-baseline --math "$MATH" --batch "$B" "$@" > "gpurun_out/pmc_${TAG}_${WL}_$C.log" 2>&1
  rc=$?
  echo "[pmc] $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_traffic.py --fetch "gpurun_out/pmc_${TAG}_${WL}_FETCH_SIZE" \
  --write "gpurun_out/pmc_${TAG}_${WL}_WRITE_SIZE" --steps $TOTAL --label "$TAG $WL $MATH b$B $*" \
  --out "gpurun_out/pmc_${WL}_${MATH}_b$B.json"
