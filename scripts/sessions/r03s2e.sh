#!/bin/bash
# Chain Adam (depth_net buckets on its filter-gradient stream): trainer/DDP/full-size GPU tests, then A/B of TDE_C4_CHAIN_ADAM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_r03s2e.log 2>&1
rc=$?; tail -5 gpurun_out/tests_r03s2e.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 0 1; do
    TDE_C4_CHAIN_ADAM=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab_r03s2e_m${m}_$i.json 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
    echo "chain_adam=$m run $i: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03s2e_m${m}_$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
