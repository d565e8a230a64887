#!/bin/bash
# Host-knob sweep on the current tree: skinny-path row limit, fp32 MFMA for 16-wide tiles, split-K minimum
# k-tiles, BN partial-sum grain; micro-benchmarks of the affected shapes, then config-2 / config-4 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" "TDE_SKINNY_M=96" "TDE_MATH4_MIN_BN=32"; do
  echo "== micro [$v]"
  env $v timeout -k 10 120 python3 -u scripts/conv_micro.py --math fp16x3 --shapes cnv6b,cnv7,icnv7,icnv1,upcnv1,upcnv2 --modes fwd,dgrad --reps 50 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2; do
  bash scripts/ab_env.sh "base:TDE_X=0" "sk96:TDE_SKINNY_M=96" "m4bn32:TDE_MATH4_MIN_BN=32" "minkt2:TDE_SPLIT_MINKT=2" "bnel4k:TDE_BN_ELEMS=4096" "bnel16k:TDE_BN_ELEMS=16384" || exit 1
done
AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4base:TDE_X=0" "c4sk96:TDE_SKINNY_M=96" "c4m4bn32:TDE_MATH4_MIN_BN=32" "c4minkt2:TDE_SPLIT_MINKT=2" "c4bnel4k:TDE_BN_ELEMS=4096" || exit 1
