#!/bin/bash
# Pipelined k-loop (next tile's split + LDS stores between the current tile's MFMA rows; PF 2 path): parity with it
# on for every tile (TDE_PF128=2 TDE_PF64=2), kernel-level timings under rocprofv3, config-4 / config-2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TDE_PF128=2 TDE_PF64=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv or deconv" \
  --timeout 120 --timeout-method thread > gpurun_out/r03zb_tests.log 2>&1
rc=$?; echo "[r03zb] kernel tests pipe rc=$rc"; tail -1 gpurun_out/r03zb_tests.log; [ $rc -ne 0 ] && exit $rc
S=gemm1x1_big,big3x3,icnv4,icnv5,cnv4b
for v in p1 p2 p22; do
  P128=1; P64=1; [ $v = p2 ] && P128=2; [ $v = p22 ] && { P128=2; P64=2; }
  TDE_PF128=$P128 TDE_PF64=$P64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r03zb_$v" -o run \
    --output-format csv -- python3 scripts/conv_micro.py --math fp16x3 --reps 10 --shapes $S > gpurun_out/r03zb_$v.log 2>&1
  rc=$?; echo "[r03zb] micro $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03zb_$v.log; exit $rc; }
done
for r in 1 2; do
  for v in p1 p2 p22; do
    P128=1; P64=1; [ $v = p2 ] && P128=2; [ $v = p22 ] && { P128=2; P64=2; }
    TDE_PF128=$P128 TDE_PF64=$P64 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline \
      --no-secondary > gpurun_out/ab_r03zb_$v$r.json 2> gpurun_out/ab_r03zb_$v$r.err
    rc=$?; echo "[r03zb] c4 $v/$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03zb_$v$r.json')); k=d['kernel_breakdown_ms']; print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], k['conv_fwd'], k['conv_bwd'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for v in p1 p22; do
  P128=1; P64=1; [ $v = p22 ] && { P128=2; P64=2; }
  TDE_PF128=$P128 TDE_PF64=$P64 timeout -k 10 200 python bench.py --workload config2 --steps 50 --warmup 10 \
    --no-cpu-baseline --no-secondary > gpurun_out/ab_r03zb_c2_$v.json 2> gpurun_out/ab_r03zb_c2_$v.err
  rc=$?; echo "[r03zb] c2 $v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03zb_c2_$v.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "[r03zb] done"
