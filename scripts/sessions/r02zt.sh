#!/bin/bash
# Diagnostic: the failing captured net-overlap test alone, HIP log level 3 (tail kept).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AMD_LOG_LEVEL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainers.py -x -q -m gpu -k "net_overlap and graph and wgrad_inline" --timeout 240 --timeout-method thread > /tmp/hiplog.txt 2>&1
rc=$?
echo "rc=$rc"
grep -c "" /tmp/hiplog.txt
grep -v "hipGetLastError\|hip_error.cpp" /tmp/hiplog.txt | tail -300 > gpurun_out/r02zt_tail.txt
grep -n "passed\|failed\|Fatal\|Segmentation" /tmp/hiplog.txt | head
exit 0
