#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nets.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02m_tests.log
[ $rc -eq 0 ] || exit $rc
for e in "TDE_BN_SMALL_UNFUSED=1" "TDE_BN_SMALL_UNFUSED=0"; do
  env $e timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r02m_bench.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02m_bench.json'));print('$e',d['value'],d['ms_per_step'])"
done
