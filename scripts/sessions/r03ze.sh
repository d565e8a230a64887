#!/bin/bash
# Head filter gradients on the filter-gradient side stream (TDE_HEAD_WGRAD_SIDE=1, data gradient on the compute
# stream): trainer / DDP / net tests, then config-4 and config-2 A/B against the fused head backward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_nets.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/r03ze_tests.log 2>&1
rc=$?; echo "[r03ze] tests rc=$rc"; tail -1 gpurun_out/r03ze_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 0 1; do
    TDE_HEAD_WGRAD_SIDE=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r03ze_h$v$r.json 2> gpurun_out/ab_r03ze_h$v$r.err
    rc=$?; echo "[r03ze] c4 head_side=$v/$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03ze_h$v$r.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for v in 0 1; do
  TDE_HEAD_WGRAD_SIDE=$v timeout -k 10 200 python bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline \
    --no-secondary > gpurun_out/ab_r03ze_c2_h$v.json 2> gpurun_out/ab_r03ze_c2_h$v.err
  rc=$?; echo "[r03ze] c2 head_side=$v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03ze_c2_h$v.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "[r03ze] done"
