#!/bin/bash
# Round 4: halo-conv threshold 8192 output pixels as the default -- conv / trainer / full-size GPU tests, then the
# default against the old threshold (TDE_HALO_MIN_M=16384), alternating x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp AB_BENCH_ARGS="--no-secondary"
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainers.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04z2.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r04z2.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  bash scripts/ab_env.sh "new$rep:TDE_HALO_MIN_M=8192" "old$rep:TDE_HALO_MIN_M=16384" || exit $?
done
