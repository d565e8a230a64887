# Round 6: the stride-2 halo filter gradient -- kernel tests, per-layer A/B over TDE_HWH_S2_MAXC, config-4 bench.
# Usage: r06_hwh2.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06h}
out=gpurun_out/hwh2_${tag}.txt
: > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread \
  -k "halo_stride2 or fp16x3_operand_bounds or pixel_shuffle or conv2d_fwd_bwd" >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -3 $out
for mc in 0 8 16; do
  echo "== TDE_HWH_S2_MAXC=$mc" >> $out
  TDE_HWH_S2_MAXC=$mc timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes wgrad --reps 30 \
    --shapes cnv1c4_b16,cnv1p_b16,upcnv1_b16,expup1_b16 >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "^\.\|passed" $out | tail -20
for mc in 0 8; do
  TDE_HWH_S2_MAXC=$mc timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${tag}_mc${mc}.json 2> gpurun_out/bench_${tag}_mc${mc}.err || { tail -20 gpurun_out/bench_${tag}_mc${mc}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_mc${mc}.json mc$mc
done
