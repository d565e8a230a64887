#!/bin/bash
# Shuffle row-lane combine in the BN / split-K partial-sum kernels: tests, then same-box A/B against the
# previous finalize (variants/libtde_prev.so) on configs 2 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nets.py tests/test_gpu_trainers.py -x -q -m gpu -k "bn or BN or batch or net or step or trainer or sync" --timeout 120 --timeout-method thread > gpurun_out/r02zi_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02zi_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for WL in config2 config4; do
for lib in tf_depth_estimation_amd/libtde.so variants/libtde_prev.so; do
  TDE_LIBRARY=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $WL --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/r02zi_b.json 2>gpurun_out/r02zi_b.err || { tail -5 gpurun_out/r02zi_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02zi_b.json'));print('$WL $lib',d['value'],d['ms_per_step'],d['kernel_breakdown_ms']['bn_fwd'],d['kernel_breakdown_ms']['bn_bwd'])"
done
done
done
