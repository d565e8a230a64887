#!/bin/bash
# Diagnostic of the capture_end segfault with the config-4 net overlap: HIP log level 3 of one capture.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AMD_LOG_LEVEL=3 timeout -k 10 120 python -u probe/net_overlap_capture.py > /tmp/hiplog.txt 2>&1
rc=$?
echo "rc=$rc"
grep -n "capturing\|captured\|replayed" /tmp/hiplog.txt | head
grep -c "" /tmp/hiplog.txt
tail -400 /tmp/hiplog.txt > gpurun_out/r02zs_tail.txt
grep -n -i "error\|fail" /tmp/hiplog.txt | tail -40 > gpurun_out/r02zs_err.txt
exit 0
