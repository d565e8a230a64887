#!/bin/bash
# Deep layers' filter gradients inline (fused data + filter gradient launch on the compute stream) instead of on
# the side stream: TDE_WGRAD_INLINE_M thresholds, config-2 / config-4 benches, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  bash scripts/ab_env.sh "base:TDE_X=0" "in96:TDE_WGRAD_INLINE_M=96" "in384:TDE_WGRAD_INLINE_M=384" "in1536:TDE_WGRAD_INLINE_M=1536" "in6144:TDE_WGRAD_INLINE_M=6144" || exit 1
done
AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4base:TDE_X=0" "c4in384:TDE_WGRAD_INLINE_M=384" "c4in1536:TDE_WGRAD_INLINE_M=1536" "c4in6144:TDE_WGRAD_INLINE_M=6144" || exit 1
