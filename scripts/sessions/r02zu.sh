#!/bin/bash
# Diagnostic: the trainer test file up to the captured net-overlap test, HIP error log (level 1), no capture.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AMD_LOG_LEVEL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py -x -q -s -m gpu -k "not rejects" --timeout 120 --timeout-method thread > /tmp/t.txt 2>&1
rc=$?
echo "rc=$rc"
grep -v "^\s*$" /tmp/t.txt | grep -v "_pytest\|pluggy" | tail -60 > gpurun_out/r02zu_tail.txt
grep -n ":1:\|rror" /tmp/t.txt | head -40 > gpurun_out/r02zu_err.txt
exit 0
