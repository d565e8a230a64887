#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_utils_lr.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r02c_tests.log
[ $rc -le 1 ] || exit $rc
bash scripts/sessions/r02_floor.sh
