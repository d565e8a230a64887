#!/bin/bash
# Deep-level 64-row tiles: prefetch depth 2 (2 waves/SIMD, 187 VGPR+AGPR) vs 1 (3 waves/SIMD), with split-K
# targets; conv micro-benchmarks of the deep shapes, then config-2 / config-4 benches, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" "TDE_CONV_PF=1" "TDE_CONV_PF=1 TDE_SPLIT_TARGET=768"; do
  echo "== micro [$v]"
  env $v timeout -k 10 120 python3 -u scripts/conv_micro.py --math fp16x3 --shapes icnv5,icnv6,cnv4b,cnv6b,upcnv5,upcnv6 --modes fwd,dgrad --reps 50 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2; do
  bash scripts/ab_env.sh "base:TDE_X=0" "pf1:TDE_CONV_PF=1" "pf1t768:TDE_CONV_PF=1 TDE_SPLIT_TARGET=768" || exit 1
  AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4base:TDE_X=0" "c4pf1:TDE_CONV_PF=1" "c4pf1t768:TDE_CONV_PF=1 TDE_SPLIT_TARGET=768" || exit 1
done
