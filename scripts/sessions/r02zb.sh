#!/bin/bash
# Deferred Adam (optimizer step overlapped with the next forward) + lazy per-bucket weight splits: trainer / ddp /
# net / inference GPU tests, then an A/B bench of --deferred-adam on/off on configs 2 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r02zb
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_nets.py tests/test_gpu_inference.py tests/test_gpu_checkpoint.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for WL in config2 config4; do
for d in off on; do
  timeout -k 10 200 python -u bench.py --workload $WL --steps 30 --warmup 10 --no-cpu-baseline --deferred-adam $d > gpurun_out/${TAG}_b.json 2>gpurun_out/${TAG}_b.err || { tail -5 gpurun_out/${TAG}_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_b.json'));print('$WL deferred $d',d['value'],d['ms_per_step'])"
done
done
done
