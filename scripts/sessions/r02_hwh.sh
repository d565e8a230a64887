#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv or deconv" --timeout 120 --timeout-method thread > gpurun_out/r02_hwh_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r02_hwh_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/conv_micro.py --math fp16x3 --reps 20 --modes wgrad --shapes cnv1b,icnv1,icnv2,cnv2b,icnv3 > gpurun_out/r02_micro_hwh.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r02_micro_hwh.log
[ $rc -eq 0 ] || exit $rc
TDE_HWH=0 timeout -k 10 300 python -u scripts/conv_micro.py --math fp16x3 --reps 20 --modes wgrad --shapes cnv1b,icnv1,icnv2 > gpurun_out/r02_micro_hwh0.log 2>&1
echo "micro0 rc=$?"; cat gpurun_out/r02_micro_hwh0.log
