#!/bin/bash
# Round 4: the halo conv threshold lowered further (4096 / 6144 output pixels) -- the conv / trainer / full-size GPU
# tests under TDE_HALO_MIN_M=4096 first, then the bench alternating x3 against the default 8192.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp AB_BENCH_ARGS="--no-secondary"
TDE_HALO_MIN_M=4096 timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainers.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04zx.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r04zx.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  bash scripts/ab_env.sh "base$rep:TDE_HALO_MIN_M=8192" "halo4k$rep:TDE_HALO_MIN_M=4096" "halo6k$rep:TDE_HALO_MIN_M=6144" || exit $?
done
