#!/bin/bash
# Two-chain config-4 schedule (one join): trainer/DDP/full-size GPU tests, then config-4 A/B of TDE_C4_CHAINS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_r03s2d.log 2>&1
rc=$?; tail -5 gpurun_out/tests_r03s2d.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 0 1; do
    TDE_C4_CHAINS=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab_r03s2d_m${m}_$i.json 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
    echo "chains=$m run $i: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03s2d_m${m}_$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
