#!/bin/bash
# Where the implicit-GEMM k-loop time goes: the same micro shapes with one phase removed per build
# (variants/libtde_dbg{1,2,3}.so: 1 no global loads, 2 no MFMAs, 3 no split/LDS staging; timings only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
S=gemm1x1_big,big3x3,cnv1b,icnv4,icnv5,cnv4b
for v in base dbg1 dbg2 dbg3; do
  L=$PWD/tf_depth_estimation_amd/libtde.so; [ $v != base ] && L=$PWD/variants/libtde_$v.so
  TDE_LIBRARY=$L timeout -k 10 200 python scripts/conv_micro.py --math fp16x3 --reps 20 --shapes $S \
    > gpurun_out/r03p_micro_$v.txt 2>&1
  rc=$?; echo "[r03p] micro $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03p_micro_$v.txt; exit $rc; }
done
echo "[r03p] done"
