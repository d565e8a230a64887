# Round 6: stride-2 halo filter gradient (8-16 channel views) -- tests, per-layer table, bench A/B against off.
# Usage: r06_hwh4.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06l}
out=gpurun_out/hwh4_${tag}.txt
: > $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_trainers.py -x -q \
  --timeout 150 --timeout-method thread -k "halo or fp16x3_operand_bounds or pixel_shuffle or conv2d_fwd_bwd or deconv or config4 or config3" >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -3 $out
for mc in 0 16; do
  echo "== TDE_HWH_S2_MAXC=$mc" >> $out
  TDE_HWH_S2_MAXC=$mc timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes wgrad --reps 30 \
    --shapes cnv1c4_b16,cnv1p_b16,upcnv1_b16,expup1_b16 >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "^\.\|passed\|amdgpu.ids" $out | tail -12
n=0
for v in 0 16 0 16; do
  n=$((n+1))
  TDE_HWH_S2_MAXC=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/bench_${tag}_mc${v}_$n.json 2> gpurun_out/bench_${tag}_mc${v}_$n.err || { tail -20 gpurun_out/bench_${tag}_mc${v}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_mc${v}_$n.json "mc$v"
done
