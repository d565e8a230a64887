#!/bin/bash
# Round 2 session 7 final check of the committed tree: all GPU tests, smoke(), the four benches, and a
# rocprofv3 kernel-trace summary of the default bench (config 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/final_smoke.log; [ $rc -ne 0 ] && exit $rc
STEPS=100 bash scripts/bench_all.sh ${TAG:-r02s7} || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG:-r02s7}_config2" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG:-r02s7}_config2.log 2>&1 || exit 1
find gpurun_out/prof_${TAG:-r02s7}_config2 -name "*stats*"
