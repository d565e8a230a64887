#!/bin/bash
# Round 4: BN partial-pass block size and split-K block target re-checked after the small-BN threshold moved to 512
# (same box, alternating x2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AB_BENCH_ARGS="--no-secondary"
for rep in 1 2; do
  bash scripts/ab_env.sh "base$rep:TDE_BN_ELEMS=8192" "elems4k$rep:TDE_BN_ELEMS=4096" "elems16k$rep:TDE_BN_ELEMS=16384" \
    "split320_$rep:TDE_SPLIT_TARGET=320" "split448_$rep:TDE_SPLIT_TARGET=448" || exit $?
done
