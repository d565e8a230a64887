#!/bin/bash
# HBM traffic AND MFMA-pipe busy of one bench workload, per kernel family, from three separate rocprofv3
# counter passes over the same eager bench command (counters cannot share a pass: FETCH_SIZE uses 3 of the 4
# TCC slots, WRITE_SIZE 2):
#   1. SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE   2. FETCH_SIZE   3. WRITE_SIZE
#   bash scripts/pmc_step.sh TAG [WORKLOAD] [MATH] [BATCH] [extra bench args]
# -> gpurun_out/pmc_<WORKLOAD>_<MATH>_b<BATCH>.json (copy to profiles/ for bench.py's roofline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
WL=${2:-config4}
MATH=${3:-fp16x3}
B=${4:-$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(bench.WORKLOADS['$WL'][2])")}
shift $(( $# < 4 ? $# : 4 ))
STEPS=4; WARM=1
# bench.py --no-graph runs 2 eager steps before the timed loop (plain + instrumented)
TOTAL=$((STEPS + WARM + 2))
i=0
for C in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d "$PWD/gpurun_out/pmc_${TAG}_${WL}_p$i" -o run \
    --output-format csv -- python3 bench.py --workload "$WL" --steps $STEPS --warmup $WARM --no-graph \
    --no-cpu-baseline --no-secondary --math "$MATH" --batch "$B" "$@" > "gpurun_out/pmc_${TAG}_${WL}_p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_traffic.py --sq "gpurun_out/pmc_${TAG}_${WL}_p1" --fetch "gpurun_out/pmc_${TAG}_${WL}_p2" \
  --write "gpurun_out/pmc_${TAG}_${WL}_p3" --steps $TOTAL --label "$TAG $WL $MATH b$B $*" \
  --out "gpurun_out/pmc_${WL}_${MATH}_b$B.json" > /dev/null
rc=$?
[ $rc -eq 0 ] && rm -rf "gpurun_out/pmc_${TAG}_${WL}_p1" "gpurun_out/pmc_${TAG}_${WL}_p2" "gpurun_out/pmc_${TAG}_${WL}_p3"
exit $rc
