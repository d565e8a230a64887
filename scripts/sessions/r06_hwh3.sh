# Round 6: XCD-grouped halo filter gradient -- kernel tests, per-layer A/B (TDE_HWH_XCD x TDE_HWH_S2_MAXC), bench.
# Usage: r06_hwh3.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06k}
out=gpurun_out/hwh3_${tag}.txt
: > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread \
  -k "halo_stride2 or fp16x3_operand_bounds or conv2d_fwd_bwd" >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -3 $out
for xcd in 0 1; do
  for mc in 8 16; do
    echo "== TDE_HWH_XCD=$xcd TDE_HWH_S2_MAXC=$mc" >> $out
    TDE_HWH_XCD=$xcd TDE_HWH_S2_MAXC=$mc timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes wgrad \
      --reps 30 --shapes cnv1c4_b16,cnv1p_b16,upcnv1_b16,expup1_b16,cnv1b,icnv1,icnv2,icnv2_b16 >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
grep -v "^\.\|passed\|amdgpu.ids" $out | tail -44
for v in "0 8" "1 8" "1 16"; do
  set -- $v
  TDE_HWH_XCD=$1 TDE_HWH_S2_MAXC=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${tag}_x$1_mc$2.json 2> gpurun_out/bench_${tag}_x$1_mc$2.err || { tail -20 gpurun_out/bench_${tag}_x$1_mc$2.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_x$1_mc$2.json "xcd$1 mc$2"
done
