#!/bin/bash
# Per-layer dz buffers + grouped side-stream forks (TDE_WGRAD_GROUP): trainer/ddp tests, then a bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/wgg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/wgg_tests.log
[ $rc -eq 0 ] || exit $rc
for WL in ${WLS:-config2}; do
for g in ${GROUPS_:-1 2 3 4 6}; do
  TDE_WGRAD_GROUP=$g timeout -k 10 200 python -u bench.py --workload $WL --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/wgg_bench.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/wgg_bench.json'));print('$WL group $g',d['value'],d['ms_per_step'])"
done
done
