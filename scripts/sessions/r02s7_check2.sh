#!/bin/bash
# Pyramid block cap 192 (new default) vs 128: all GPU tests, alternating config-2 / config-4 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/check2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/check2_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_env.sh "m192:TDE_X=0" "m128:TDE_PYR_MAXB=128" "m192b:TDE_X=0" "m128b:TDE_PYR_MAXB=128" || exit 1
AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4m192:TDE_X=0" "c4m128:TDE_PYR_MAXB=128" "c4m192b:TDE_X=0" "c4m128b:TDE_PYR_MAXB=128" || exit 1
