# Round 6: fp16x3 GEMM tiles allocated for 3 waves per SIMD (TDE_GEMM_WAVES=3, in-tree) vs the previous allocation
# (libtde_w1.so, -DTDE_GEMM_WAVES=1): conv tests, per-layer times, bench alternating.  Usage: r06_gemmwaves.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06y}
out=gpurun_out/gemmwaves_${tag}.txt
: > $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -2 $out
W1=$PWD/tf_depth_estimation_amd/libtde_w1.so
SH=cnv2_b16,cnv3_b16,cnv4_b16,cnv3b_b16,cnv4b_b16,icnv4_b16,icnv5_b16,upcnv2_b16,upcnv3_b16,cnv2b_b16
for v in new old; do
  echo "== $v" >> $out
  if [ $v = old ]; then export TDE_LIBRARY=$W1; else unset TDE_LIBRARY; fi
  timeout -k 10 200 python -u scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad,wgrad --reps 20 --shapes $SH >> $out 2>&1 || { tail -20 $out; exit 1; }
done
unset TDE_LIBRARY
grep -v "^\.\|passed\|amdgpu.ids" $out
n=0
for v in old new old new; do
  n=$((n+1))
  if [ $v = old ]; then export TDE_LIBRARY=$W1; else unset TDE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary > gpurun_out/bench_${tag}_${v}_$n.json 2> gpurun_out/bench_${tag}_${v}_$n.err || { tail -20 gpurun_out/bench_${tag}_${v}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_${v}_$n.json "$v"
done
