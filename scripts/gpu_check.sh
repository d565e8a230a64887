#!/bin/bash
# One GPU-box session: parity tests, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault / abort / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
STEPS=${STEPS:-50}
WL=${WL:-config2}

ok_or_stop() {  # rc 0 (pass) and 1 (test failures) keep going; anything else is a fault/timeout
  local rc=$1 what=$2
  echo "[gpu_check] $what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_check] stopping after $what"; exit "$rc"; fi
}

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${TESTS:-} > gpurun_out/gpu_tests.log 2>&1
  ok_or_stop $? "pytest -m gpu"
  grep -E "passed|failed|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -20
fi

if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 400 python bench.py --workload "$WL" --steps "$STEPS" --warmup 10 ${BENCH_ARGS:-} \
    > gpurun_out/bench_${TAG}_$WL.json 2> gpurun_out/bench_${TAG}_$WL.err
  ok_or_stop $? "bench"
  cat gpurun_out/bench_${TAG}_$WL.json
fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_$WL" -o run --output-format csv \
    -- python3 bench.py --workload "$WL" --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/prof_${TAG}_$WL.log 2>&1
  ok_or_stop $? "rocprofv3"
  find gpurun_out/prof_${TAG}_$WL -name "*stats*"
fi
