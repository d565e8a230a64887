#!/bin/bash
# Profile the current tree's default bench (config 4): kernel trace (per-queue step summary) and the PMC passes
# (MFMA busy + HBM traffic per family) for bench.py's roofline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03q
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_config4" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/prof_${TAG}_config4.log 2>&1
rc=$?; echo "[r03q] trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/queue_summary.py gpurun_out/prof_${TAG}_config4/run_kernel_trace.csv 40 > gpurun_out/${TAG}_config4_step_by_queue.txt
echo "[r03q] queue summary rc=$?"
bash scripts/pmc_step.sh $TAG config4 fp16x3 8
echo "[r03q] pmc rc=$?"
