#!/bin/bash
# XCD-contiguous channel-quad blocks in the per-quad BatchNorm kernels (TDE_BN_XCD, bn.hip) vs hardware order
# (variants/libtde_bnx0.so): BN/trainer GPU tests, alternating config-2 / config-4 benches, and a rocprofv3
# kernel-trace summary of each build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
X0="TDE_LIBRARY=$PWD/variants/libtde_bnx0.so"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainers.py -q -m gpu -k "bn or BN or Bn or config" \
  --timeout 120 --timeout-method thread > gpurun_out/bnxcd_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bnxcd_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  bash scripts/ab_env.sh "x1_$r:TDE_X=0" "x0_$r:$X0" || exit 1
done
AB_BENCH_ARGS="--workload config4" bash scripts/ab_env.sh "c4x1:TDE_X=0" "c4x0:$X0" "c4x1b:TDE_X=0" "c4x0b:$X0" || exit 1
for v in x1 x0; do
  if [ $v = x0 ]; then export TDE_LIBRARY=$PWD/variants/libtde_bnx0.so; else unset TDE_LIBRARY; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_bn$v" -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bn$v.log 2>&1 || exit 1
done
unset TDE_LIBRARY
for v in x1 x0; do
  f=$(find gpurun_out/prof_bn$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bn_' in r['Name'] or 'splitk_reduce_bn' in r['Name']:
        print('%10.2f us avg %6s calls  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:60]))
" "$f"
done
