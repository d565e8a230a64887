#!/bin/bash
# Pixel-shuffle deconv forward (MODE_PS): kernel parity with it forced on every eligible shape
# (TDE_DECONV_PS_MINM=1) and at the default threshold through the nets, micro-benchmarks of the deconv layers
# with it off / on, config-4 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TDE_DECONV_PS_MINM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv or deconv" \
  --timeout 120 --timeout-method thread > gpurun_out/r03x_tests_ps1.log 2>&1
rc=$?; echo "[r03x] kernel tests ps-forced (r03y) rc=$rc"; tail -1 gpurun_out/r03x_tests_ps1.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_nets.py tests/test_gpu_fullsize.py tests/test_gpu_inference.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/r03x_tests_nets.log 2>&1
rc=$?; echo "[r03x] nets/fullsize/inference rc=$rc"; tail -1 gpurun_out/r03x_tests_nets.log; [ $rc -ne 0 ] && exit $rc
S=upcnv1,upcnv2,upcnv3,upcnv1_b16,upcnv2_b16,upcnv3_b16
for v in 0 1; do
  TDE_DECONV_PS_MINM=$v timeout -k 10 200 python scripts/conv_micro.py --math fp16x3 --reps 20 --modes dgrad --shapes $S \
    > gpurun_out/r03x_micro_ps$v.txt 2>&1
  rc=$?; echo "[r03x] micro ps$v rc=$rc"; grep -v "amdgpu\|==" gpurun_out/r03x_micro_ps$v.txt; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for v in 0 8192; do
    TDE_DECONV_PS_MINM=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r03x_ps$v$r.json 2> gpurun_out/ab_r03x_ps$v$r.err
    rc=$?; echo "[r03x] c4 ps$v/$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03x_ps$v$r.json')); k=d['kernel_breakdown_ms']; print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], k['conv_fwd'], k['conv_bwd'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for v in 0 8192; do
  TDE_DECONV_PS_MINM=$v timeout -k 10 200 python bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline \
    --no-secondary > gpurun_out/ab_r03x_c2_ps$v.json 2> gpurun_out/ab_r03x_c2_ps$v.err
  rc=$?; echo "[r03x] c2 ps$v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03x_c2_ps$v.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "[r03x] done"
