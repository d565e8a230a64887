#!/bin/bash
# copy_view_kernel with 32-bit index math (adam_util.hip) vs the 64-bit version (variants/libtde_cv0.so):
# all GPU tests, rocprofv3 kernel time on config 4, alternating config-4 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cv_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cv_tests.log; [ $rc -ne 0 ] && exit $rc
fi
bash scripts/knob_kernel_sweep.sh TDE_LIBRARY copy_view "config4" "$PWD/tf_depth_estimation_amd/libtde.so $PWD/variants/libtde_cv0.so" || exit 1
X0="TDE_LIBRARY=$PWD/variants/libtde_cv0.so"
AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4cv1:TDE_X=0" "c4cv0:$X0" "c4cv1b:TDE_X=0" "c4cv0b:$X0" || exit 1
