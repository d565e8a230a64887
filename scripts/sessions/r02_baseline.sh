#!/bin/bash
# Round-2 baseline on a fresh box: GPU parity tests, conv micro-benchmark (current math), short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02_gpu_tests.log
[ $rc -le 1 ] || exit $rc
[ "${SKIP_MICRO:-0}" = "1" ] || timeout -k 10 300 python -u scripts/conv_micro.py --math bf16x6r,fp16x3 --reps 20 > gpurun_out/r02_micro_base.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r02_micro_base.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r02_bench_base.json 2> gpurun_out/r02_bench_base.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r02_bench_base.json
exit $rc
