#!/bin/bash
# Which of the two staging changes pays: v_fma_mix fp16 split (mix) and the WGRAD row-of-4 decode (row4), as
# kernel-build variants on one box (variants/libtde_{old,mixonly,row4only}.so; the tree's libtde.so = both);
# the gradient-bound pre-pass now runs on up to 1024 blocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_abi.py -q -x -k "conv or deconv or halo or bound" \
  --timeout 120 --timeout-method thread > gpurun_out/r03m_tests.log 2>&1
rc=$?; echo "[r03m] kernel tests rc=$rc"; tail -2 gpurun_out/r03m_tests.log; [ $rc -ne 0 ] && exit $rc
lib() { [ $1 = both ] && echo $PWD/tf_depth_estimation_amd/libtde.so || echo $PWD/variants/libtde_$1.so; }
for v in old mixonly row4only both; do
  TDE_LIBRARY=$(lib $v) timeout -k 10 200 python scripts/conv_micro.py --math fp16x3 --reps 20 \
    --shapes gemm1x1_big,big3x3,cnv1b,cnv2b,icnv3,icnv4,icnv5,cnv4b,cnv7,upcnv1,upcnv3 > gpurun_out/r03m_micro_$v.txt 2>&1
  rc=$?; echo "[r03m] micro $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03m_micro_$v.txt; exit $rc; }
done
for r in 1 2; do
  for v in old mixonly row4only both; do
    TDE_LIBRARY=$(lib $v) timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r03m_$v$r.json 2> gpurun_out/ab_r03m_$v$r.err
    rc=$?; echo "[r03m] bench $v$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03m_$v$r.json')); k=d['kernel_breakdown_ms']; print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], k['conv_fwd'], k['conv_bwd'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
