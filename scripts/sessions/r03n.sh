#!/bin/bash
# Row-of-4 WGRAD decode as a block-level template choice (no branch in the k-loop) vs the mix-only kernels
# (variants/libtde_mixonly.so), and the XCD-grouped WGRAD tile order (TDE_XCD_WGRAD=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv or deconv or halo" \
  --timeout 120 --timeout-method thread > gpurun_out/r03n_tests.log 2>&1
rc=$?; echo "[r03n] kernel tests rc=$rc"; tail -2 gpurun_out/r03n_tests.log; [ $rc -ne 0 ] && exit $rc
TDE_XCD_WGRAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv2d_fwd_bwd or deconv2d_fwd_bwd or bwd_fused" \
  --timeout 120 --timeout-method thread > gpurun_out/r03n_tests_xcd.log 2>&1
rc=$?; echo "[r03n] kernel tests xcd rc=$rc"; tail -2 gpurun_out/r03n_tests_xcd.log; [ $rc -ne 0 ] && exit $rc
NEW=$PWD/tf_depth_estimation_amd/libtde.so; OLD=$PWD/variants/libtde_mixonly.so
S=gemm1x1_big,big3x3,cnv1b,cnv2b,icnv3,icnv4,icnv5,cnv4b,cnv7,upcnv1,upcnv3
for v in old new xcd; do
  L=$NEW; [ $v = old ] && L=$OLD; X=0; [ $v = xcd ] && X=1
  TDE_XCD_WGRAD=$X TDE_LIBRARY=$L timeout -k 10 200 python scripts/conv_micro.py --math fp16x3 --reps 20 --modes wgrad \
    --shapes $S > gpurun_out/r03n_micro_$v.txt 2>&1
  rc=$?; echo "[r03n] micro $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03n_micro_$v.txt; exit $rc; }
done
for r in 1 2; do
  for v in old new xcd; do
    L=$NEW; [ $v = old ] && L=$OLD; X=0; [ $v = xcd ] && X=1
    TDE_XCD_WGRAD=$X TDE_LIBRARY=$L timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline \
      --no-secondary > gpurun_out/ab_r03n_$v$r.json 2> gpurun_out/ab_r03n_$v$r.err
    rc=$?; echo "[r03n] bench $v$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03n_$v$r.json')); k=d['kernel_breakdown_ms']; print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], k['conv_fwd'], k['conv_bwd'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo "[r03n] done"
