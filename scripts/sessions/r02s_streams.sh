#!/bin/bash
# Filter gradients over TDE_WGRAD_STREAMS side streams: trainer tests at 2 streams, then a bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TDE_WGRAD_STREAMS=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py -x -q -m gpu -k "not wgrad]" --timeout 120 --timeout-method thread > gpurun_out/st_tests.log 2>&1
rc=$?; echo "tests(2 streams) rc=$rc"; tail -2 gpurun_out/st_tests.log
[ $rc -eq 0 ] || exit $rc
for WL in ${WLS:-config2 config4}; do
for r in 1 2; do
for n in ${NS:-1 2 3}; do
  TDE_WGRAD_STREAMS=$n timeout -k 10 200 python -u bench.py --workload $WL --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/sb.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sb.json'));print('$WL streams $n',d['value'],d['ms_per_step'])"
done
done
done
