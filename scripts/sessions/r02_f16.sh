#!/bin/bash
# fp16x3 (conv math 4) prototype: kernel parity + micro-benchmark against bf16x6r.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv or deconv" --timeout 120 --timeout-method thread > gpurun_out/r02_f16_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r02_f16_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/conv_micro.py --math bf16x6r,fp16x3 --reps 20 > gpurun_out/r02_micro_f16.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r02_micro_f16.log
[ $rc -eq 0 ] || exit $rc
TDE_MATH4_MIN_BN=64 timeout -k 10 300 python -u scripts/conv_micro.py --math fp16x3 --reps 20 --shapes icnv1,icnv2,cnv1b,cnv2b,icnv3 > gpurun_out/r02_micro_f16_nar.log 2>&1
echo "micro64 rc=$?"; cat gpurun_out/r02_micro_f16_nar.log
