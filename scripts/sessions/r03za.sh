#!/bin/bash
# Phase-removal builds of the igemm k-loop (bit mask: 1 no loads, 2 no MFMAs, 4 no staging; timings only), kernel
# time from a rocprofv3 kernel trace (excludes the bound pre-pass and the split-K reduce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=gemm1x1_big,big3x3,icnv4,icnv5,cnv4b
for v in base dbg1 dbg4 dbg5 dbg7; do
  L=$PWD/tf_depth_estimation_amd/libtde.so; [ $v != base ] && L=$PWD/variants/libtde_$v.so
  TDE_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r03za_$v" -o run \
    --output-format csv -- python3 scripts/conv_micro.py --math fp16x3 --reps 10 --shapes $S > gpurun_out/r03za_$v.log 2>&1
  rc=$?; echo "[r03za] $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03za_$v.log; exit $rc; }
done
echo "[r03za] done"
