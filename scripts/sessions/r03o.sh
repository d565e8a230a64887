#!/bin/bash
# Two k-tiles in flight for the 128-row conv tiles (TDE_PF128=2, now capped at 256 VGPRs = the 2 waves per SIMD
# those tiles already run at) vs one (default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pf in 1 2; do
  TDE_PF128=$pf timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv or deconv" \
    --timeout 120 --timeout-method thread > gpurun_out/r03o_tests_pf$pf.log 2>&1
  rc=$?; echo "[r03o] kernel tests pf$pf rc=$rc"; tail -1 gpurun_out/r03o_tests_pf$pf.log; [ $rc -ne 0 ] && exit $rc
done
S=gemm1x1_big,big3x3,cnv1b,cnv2b,icnv3,icnv4,icnv5,cnv4b,upcnv1,upcnv3
for pf in 1 2; do
  TDE_PF128=$pf timeout -k 10 200 python scripts/conv_micro.py --math fp16x3 --reps 20 --shapes $S \
    > gpurun_out/r03o_micro_pf$pf.txt 2>&1
  rc=$?; echo "[r03o] micro pf$pf rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03o_micro_pf$pf.txt; exit $rc; }
done
for r in 1 2; do
  for pf in 1 2; do
    TDE_PF128=$pf timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline \
      --no-secondary > gpurun_out/ab_r03o_pf$pf$r.json 2> gpurun_out/ab_r03o_pf$pf$r.err
    rc=$?; echo "[r03o] bench pf$pf$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03o_pf$pf$r.json')); k=d['kernel_breakdown_ms']; print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], k['conv_fwd'], k['conv_bwd'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for pf in 1 2; do
  TDE_PF128=$pf timeout -k 10 200 python bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline \
    --no-secondary > gpurun_out/ab_r03o_c2_pf$pf.json 2> gpurun_out/ab_r03o_c2_pf$pf.err
  rc=$?; echo "[r03o] bench c2 pf$pf rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03o_c2_pf$pf.json')); print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "[r03o] done"
