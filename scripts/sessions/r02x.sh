#!/bin/bash
# Loss-head launch consolidation (arena zeroing, multi-scale pyramid loss, in-place output gradients) for
# configs 3/4/5: trainer / ddp / net GPU tests, then the four workloads' bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02x}
timeout -k 10 500 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_nets.py tests/test_gpu_utils_lr.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for WL in ${WLS:-config2 config3 config4 config5}; do
  timeout -k 10 200 python -u bench.py --workload $WL --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_$WL.json 2>gpurun_out/${TAG}_$WL.err || { tail -5 gpurun_out/${TAG}_$WL.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$WL.json'));print('$WL',d['value'],d['ms_per_step'],d.get('depth_l1_vs_ref',{}).get('worst_max_rel'))"
done
