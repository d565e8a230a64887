#!/bin/bash
# In-place input / output gradients (config 2): trainer + net GPU tests, bench, config-4 / config-3 kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02v}
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_nets.py tests/test_gpu_ddp.py tests/test_gpu_utils_lr.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_b.json'));print('config2',d['value'],d['ms_per_step'])"
done
for WL in config4 config3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_$WL" -o run --output-format csv \
    -- python3 bench.py --workload "$WL" --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/prof_${TAG}_$WL.log 2>&1 || { echo "rocprofv3 $WL failed"; exit 1; }
  tail -1 gpurun_out/prof_${TAG}_$WL.log | cut -c1-150
done
