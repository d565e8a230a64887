#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py -x -q -m gpu -k "adam_overlap or wgrad" --timeout 120 --timeout-method thread > gpurun_out/r02l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02l_tests.log
[ $rc -eq 0 ] || exit $rc
for args in "--adam-overlap off" "--adam-overlap wgrad" "--adam-overlap wgrad --adam-bucket-mb 4" "--adam-overlap side"; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline $args > gpurun_out/r02l_bench.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02l_bench.json'));print('$args',d['value'],d['ms_per_step'])"
done
