#!/bin/bash
# Round 4: path-selection thresholds re-checked under the two-chain schedule (halo conv / halo filter-gradient
# grid / pixel-shuffle deconv), same box, alternating x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AB_BENCH_ARGS="--no-secondary"
for rep in 1 2; do
  bash scripts/ab_env.sh "base$rep:TDE_HALO_MIN_M=16384" "halo8k$rep:TDE_HALO_MIN_M=8192" "halo32k$rep:TDE_HALO_MIN_M=32768" \
    "hwg512_$rep:TDE_HWG_BLOCKS=512" "hwg1024_$rep:TDE_HWG_BLOCKS=1024" "ps4k$rep:TDE_DECONV_PS_MINM=4096" \
    "ps16k$rep:TDE_DECONV_PS_MINM=16384" || exit $?
done
