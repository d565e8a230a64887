#!/bin/bash
# Write-through (sc1) epilogue stores of the implicit-GEMM conv (TDE_WT bit 0: split-K slabs, bit 1: direct
# outputs): conv kernel parity with them on, then config 4 / config 2 A/B on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TDE_WT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv or deconv" \
  --timeout 120 --timeout-method thread > gpurun_out/r03v_tests.log 2>&1
rc=$?; echo "[r03v] kernel tests wt=3 rc=$rc"; tail -1 gpurun_out/r03v_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for wt in 0 1 3; do
    TDE_WT=$wt timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r03v_wt$wt$r.json 2> gpurun_out/ab_r03v_wt$wt$r.err
    rc=$?; echo "[r03v] c4 wt$wt$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03v_wt$wt$r.json')); k=d['kernel_breakdown_ms']; print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for wt in 0 3; do
  TDE_WT=$wt timeout -k 10 200 python bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline \
    --no-secondary > gpurun_out/ab_r03v_c2_wt$wt.json 2> gpurun_out/ab_r03v_c2_wt$wt.err
  rc=$?; echo "[r03v] c2 wt$wt rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03v_c2_wt$wt.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "[r03v] done"
