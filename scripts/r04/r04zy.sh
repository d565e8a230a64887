#!/bin/bash
# Round 4: more path thresholds under the two-chain schedule (halo filter gradient from N*H*W, 64-row tile limit,
# head tiling), same box, alternating x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AB_BENCH_ARGS="--no-secondary"
for rep in 1 2; do
  bash scripts/ab_env.sh "base$rep:TDE_HWG_MIN_M=16384" "hwgm8k$rep:TDE_HWG_MIN_M=8192" "bm64_2k$rep:TDE_BM64_MAXM=2048" \
    "bm64_8k$rep:TDE_BM64_MAXM=8192" "headt16k$rep:TDE_HEAD_TILE_MIN=16384" "headt64k$rep:TDE_HEAD_TILE_MIN=65536" || exit $?
done
