#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/conv_micro.py --math bf16x3,fp32 --reps 20 --shapes gemm1x1_big,big3x3,icnv4,icnv5,icnv6,cnv4b,icnv3 > gpurun_out/r02e_micro.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r02e_micro.log
