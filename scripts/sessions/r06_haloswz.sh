# Round 6: halo conv with XOR-swizzled compact halo rows -- tests, per-layer A/B (TDE_HALO_SWZ), bench A/B.  Usage: r06_haloswz.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06w}
out=gpurun_out/haloswz_${tag}.txt
: > $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_nets.py -x -q --timeout 150 --timeout-method thread \
  -k "halo or fp16x3_operand_bounds or conv2d_fwd_bwd or split_weights or deconv" >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -2 $out
for ku in 0 1; do
  echo "== TDE_HALO_SWZ=$ku" >> $out
  TDE_HALO_SWZ=$ku timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad --reps 30 \
    --shapes cnv1b_b16,icnv1_b16,icnv2_b16,cnv2b_b16,icnv3_b16 >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "^\.\|passed\|amdgpu.ids" $out
n=0
for ku in 0 1 0 1; do
  n=$((n+1))
  TDE_HALO_SWZ=$ku timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary > gpurun_out/bench_${tag}_ku${ku}_$n.json 2> gpurun_out/bench_${tag}_ku${ku}_$n.err || { tail -20 gpurun_out/bench_${tag}_ku${ku}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_ku${ku}_$n.json "ku$ku"
done
