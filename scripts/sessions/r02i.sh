#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py -x -q -m gpu -k "wgrad or overlapped or adam_overlap" --timeout 120 --timeout-method thread > gpurun_out/r02i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r02i_tests.log
exit $rc
