#!/bin/bash
# Config-4 net overlap (depth_net on a second stream beside disp_net): trainer GPU tests, then same-box
# A/B of bench --net-overlap on/off (config 4), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_trainers.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02zq_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02zq_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for o in on off; do
    timeout -k 10 200 python -u bench.py --workload config4 --net-overlap $o --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/r02zq_b.json 2>gpurun_out/r02zq_b.err || { tail -5 gpurun_out/r02zq_b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r02zq_b.json'));print('config4 net_overlap=$o',d['value'],d['ms_per_step'],d['config']['net_overlap'], d['final_loss'])"
  done
done
