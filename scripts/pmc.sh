#!/bin/bash
# HBM traffic of one bench workload from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE), eager
# mode (the same kernels as the captured graph, one dispatch each), then the per-family summary.
#   bash scripts/pmc.sh TAG [WORKLOAD] [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=${1:-r01}
WL=${2:-config2}
shift 2 || true
STEPS=6; WARM=2
# bench.py --no-graph runs 2 eager steps before the timed loop (plain + instrumented)
TOTAL=$((STEPS + WARM + 2))
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc "$C" --kernel-trace -d "$PWD/gpurun_out/pmc_${TAG}_${WL}_$C" -o run \
    --output-format csv -- python3 bench.py --workload "$WL" --steps $STEPS --warmup $WARM --no-graph \
    --no-cpu-baseline "$@" > "gpurun_out/pmc_${TAG}_${WL}_$C.log" 2>&1
  rc=$?
  echo "[pmc] $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_traffic.py --fetch "gpurun_out/pmc_${TAG}_${WL}_FETCH_SIZE" \
  --write "gpurun_out/pmc_${TAG}_${WL}_WRITE_SIZE" --steps $TOTAL --label "$TAG $WL $*" \
  --out "gpurun_out/pmc_${TAG}_${WL}.json"
