#!/bin/bash
# Config-4 net overlap, eager only (the captured variant segfaulted in capture_end): eager tests, then
# eager bench A/B on/off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainers.py -x -q -m gpu -k "net_overlap and eager" --timeout 120 --timeout-method thread > gpurun_out/r02zr_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02zr_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for o in on off; do
    timeout -k 10 200 python -u bench.py --workload config4 --no-graph --net-overlap $o --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02zr_b.json 2>gpurun_out/r02zr_b.err || { tail -5 gpurun_out/r02zr_b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r02zr_b.json'));print('config4 eager net_overlap=$o',d['value'],d['ms_per_step'],d['config']['net_overlap'])"
  done
done
