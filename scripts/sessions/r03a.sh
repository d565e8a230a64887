#!/bin/bash
# Round 3 first GPU session: counter list, default bench (config 4 + secondary + CPU leg), PMC passes
# (MFMA busy + HBM traffic) and a kernel trace of config 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03a}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
echo "[r03a] counters rc=$?"
grep -o "SQ_[A-Z_]*MFMA[A-Z0-9_]*\|SQ_BUSY[A-Z_]*\|GRBM_GUI_ACTIVE" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_mfma.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "[r03a] bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${TAG}.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_config4" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/prof_${TAG}_config4.log 2>&1
rc=$?; echo "[r03a] trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/pmc_step.sh $TAG config4 fp16x3 8
