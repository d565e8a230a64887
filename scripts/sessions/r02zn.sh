#!/bin/bash
# Prefetch depth 1 in fp16x3 (new default): conv/net tests; then deep-level column-tile cap (TDE_DEEP_BN)
# micro-benchmarks and config-2 / config-4 benches, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nets.py tests/test_gpu_inference.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02zn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02zn_tests.log
[ $rc -eq 0 ] || exit $rc
for v in "" "TDE_DEEP_BN=64" "TDE_DEEP_BN=32"; do
  echo "== micro [$v]"
  env $v timeout -k 10 120 python3 -u scripts/conv_micro.py --math fp16x3 --shapes icnv5,icnv6,cnv4b,cnv6b,upcnv5,upcnv6 --modes fwd,dgrad --reps 50 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2; do
  bash scripts/ab_env.sh "base:TDE_X=0" "dbn64:TDE_DEEP_BN=64" "dbn32:TDE_DEEP_BN=32" || exit 1
  AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4base:TDE_X=0" "c4dbn64:TDE_DEEP_BN=64" "c4dbn32:TDE_DEEP_BN=32" || exit 1
done
