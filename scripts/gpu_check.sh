#!/bin/bash
# One GPU-box session: parity tests, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault / abort / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
STEPS=${STEPS:-50}

ok_or_stop() {  # rc 0 (pass) and 1 (test failures) keep going; anything else is a fault/timeout
  local rc=$1 what=$2
  echo "[gpu_check] $what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_check] stopping after $what"; exit "$rc"; fi
}

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
  ok_or_stop $? "pytest -m gpu"
  tail -3 gpurun_out/gpu_tests.log
fi

timeout -k 10 400 python bench.py --steps "$STEPS" --warmup 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
ok_or_stop $? "bench"
cat gpurun_out/bench_$TAG.json

if [ "${SKIP_PROF:-0}" != "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$TAG" -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
  ok_or_stop $? "rocprofv3"
  find gpurun_out/prof_$TAG -name "*stats*" | head
fi
