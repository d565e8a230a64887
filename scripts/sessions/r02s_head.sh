#!/bin/bash
# Tiled head kernels: kernel tests, net/trainer tests, then a TDE_HEAD_TILE on/off bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k head -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/head_tests.log 2>&1
rc=$?; echo "head tests rc=$rc"; tail -3 gpurun_out/head_tests.log
[ $rc -eq 0 ] || exit $rc
if [ "${FULL:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_nets.py tests/test_gpu_trainers.py tests/test_gpu_inference.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/head_tests2.log 2>&1
  rc=$?; echo "net tests rc=$rc"; tail -3 gpurun_out/head_tests2.log
  [ $rc -eq 0 ] || exit $rc
fi
for WL in ${WLS:-config2 config4}; do
for r in 1 2; do
for t in 0 1; do
  TDE_HEAD_TILE=$t timeout -k 10 200 python -u bench.py --workload $WL --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/hb.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hb.json'));print('$WL tile $t',d['value'],d['ms_per_step'], d['kernel_breakdown_ms'].get('head_fwd'), d['kernel_breakdown_ms'].get('head_bwd'))"
done
done
done
