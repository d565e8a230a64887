#!/bin/bash
# Deconv forward (DGRAD of the virtual stride-2 conv) tile exploration: planner default vs forced tiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=upcnv1,upcnv2,upcnv3,upcnv4,upcnv5,upcnv6
for v in "" "TDE_FORCE_BM=64" "TDE_FORCE_BN=32" "TDE_FORCE_BN=64" "TDE_FORCE_BM=64 TDE_FORCE_BN=64" "TDE_FORCE_BN=128" "TDE_SPLIT_TARGET=256" "TDE_SPLIT_TARGET=1024"; do
  echo "== variant [$v]"
  env $v timeout -k 10 120 python3 -u scripts/conv_micro.py --math fp16x3 --shapes $S --modes fwd,dgrad --reps 50 2>&1 | grep -v amdgpu.ids || exit 1
done
