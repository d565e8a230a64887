#!/bin/bash
# Round-3 (session 2) closing evidence of the final tree (fused pose gradient) on the final tree: full GPU suite + smoke(), the default bench line, a kernel trace of
# the default bench (per-queue summary + step timeline) and the PMC passes the bench's roofline reads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03s2x bash scripts/sessions/r03_tests.sh
rc=$?; echo "[r03s2x] tests+smoke rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r03s2x.json 2> gpurun_out/bench_r03s2x.err
rc2=$?; echo "[r03s2x] bench rc=$rc2"; head -c 400 gpurun_out/bench_r03s2x.json; echo; [ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r03s2x_config4" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/prof_r03s2x_config4.log 2>&1
rc3=$?; echo "[r03s2x] trace rc=$rc3"; [ $rc3 -ne 0 ] && exit $rc3
python3 scripts/queue_summary.py gpurun_out/prof_r03s2x_config4/run_kernel_trace.csv 40 > gpurun_out/r03s2x_config4_step_by_queue.txt
python3 scripts/step_critical.py gpurun_out/prof_r03s2x_config4/run_kernel_trace.csv 8 > gpurun_out/r03s2x_config4_step_timeline.txt
bash scripts/pmc_step.sh r03s2x config4 fp16x3 8
echo "[r03s2x] pmc rc=$?"
exit $rc
