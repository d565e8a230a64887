#!/bin/bash
# Round 4: operand-staging ablation of the implicit-GEMM conv (timing-only diagnostic builds): FWD / DGRAD per shape
# with the B operand's (weights') loads + staging removed, the A operand's, or both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in product nob noa noab; do
  lib=tf_depth_estimation_amd/libtde.so; [ $v != product ] && lib=variants/libtde_$v.so
  TDE_LIBRARY=$lib timeout -k 10 300 python scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad --reps 20 \
    > gpurun_out/micro_r04i_$v.txt 2>&1
  rc=$?; echo "[r04i] $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/micro_r04i_$v.txt; exit $rc; }
done
paste gpurun_out/micro_r04i_product.txt gpurun_out/micro_r04i_nob.txt | head -40
