#!/bin/bash
# Staged fp16x3 split: conv parity tests, micro A/B against the register-split build, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "conv or deconv" --timeout 120 --timeout-method thread > gpurun_out/r02f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r02f_tests.log
[ $rc -eq 0 ] || exit $rc
cp tf_depth_estimation_amd/libtde.so variants/libtde_stage1.so
AB_BENCH=1 bash scripts/ab_variants.sh "big3x3,gemm1x1_big,cnv2b,icnv3,icnv4,icnv5,icnv6,cnv4b,cnv7" fwd,dgrad,wgrad fp16x3
