#!/bin/bash
# Round 4: head kernels per call, row-walk vs halo-tiled (TDE_HEAD_RW=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in 1 0; do
  TDE_HEAD_RW=$v timeout -k 10 200 python scripts/head_micro.py > gpurun_out/head_micro_r04k_rw$v.txt 2>&1
  rc=$?; echo "[r04k] rw=$v rc=$rc"; cat gpurun_out/head_micro_r04k_rw$v.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
done
exit 0
