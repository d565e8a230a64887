#!/bin/bash
# One-launch BN backward for 2048 < M <= 8192 rows (bn_bwd_mid_kernel) vs partial sums + finalize + apply
# (TDE_BN_MID=0): all GPU tests, rocprofv3 BN kernel times, alternating config-2 / config-4 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/bnmid_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bnmid_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/knob_kernel_sweep.sh TDE_BN_MID bn_ "config2" "1 0" || exit 1
bash scripts/ab_env.sh "mid1:TDE_X=0" "mid0:TDE_BN_MID=0" "mid1b:TDE_X=0" "mid0b:TDE_BN_MID=0" || exit 1
AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4mid1:TDE_X=0" "c4mid0:TDE_BN_MID=0" "c4mid1b:TDE_X=0" "c4mid0b:TDE_BN_MID=0" || exit 1
