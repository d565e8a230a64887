#!/bin/bash
# fp16 split by v_fma_mix (no pair-building moves) + WGRAD row-of-4 pixel decode: conv kernel parity, conv
# micro-benchmarks and config-4 bench against the previous kernels (variants/libtde_old.so), then SQ counters
# of the big WGRAD shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "conv or deconv or halo" --timeout 120 \
  --timeout-method thread > gpurun_out/r03l_tests.log 2>&1
rc=$?; echo "[r03l] kernel tests rc=$rc"; tail -2 gpurun_out/r03l_tests.log; [ $rc -ne 0 ] && exit $rc
for lib in old new; do
  L=$PWD/tf_depth_estimation_amd/libtde.so; [ $lib = old ] && L=$PWD/variants/libtde_old.so
  TDE_LIBRARY=$L timeout -k 10 200 python scripts/conv_micro.py --math fp16x3 --reps 20 > gpurun_out/r03l_micro_$lib.txt 2>&1
  rc=$?; echo "[r03l] micro $lib rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03l_micro_$lib.txt; exit $rc; }
done
for r in 1 2; do
  for lib in old new; do
    L=$PWD/tf_depth_estimation_amd/libtde.so; [ $lib = old ] && L=$PWD/variants/libtde_old.so
    TDE_LIBRARY=$L timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r03l_${lib}$r.json 2> gpurun_out/ab_r03l_${lib}$r.err
    rc=$?; echo "[r03l] bench $lib$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03l_${lib}$r.json')); print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], d.get('kernel_breakdown_ms'))" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
MATH=fp16x3 bash scripts/conv_pmc.sh big3x3 wgrad big3x3w > gpurun_out/r03l_pmc_big3x3w.txt 2>&1
echo "[r03l] pmc rc=$?"; tail -20 gpurun_out/r03l_pmc_big3x3w.txt
