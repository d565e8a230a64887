# Round 6: the fused backward launch (igemm_bwd2) with its 64-row data-gradient tiles two in flight (TDE_BWD2_PF2=1) vs one
# (TDE_BWD2_PF2=0): GPU conv / net / fullsize tests, per-layer times, config-4 bench alternating.  Usage: r06_pf2.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06zh}
out=gpurun_out/bwd2pf2_${tag}.txt
: > $out
TDE_BWD2_PF2=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nets.py tests/test_gpu_fullsize.py tests/test_gpu_trainers.py -x -q --timeout 150 --timeout-method thread >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -2 $out
SH=cnv3b_b16,cnv4b_b16,cnv5b_b16,icnv4_b16,icnv5_b16,icnv6,cnv4_b16,upcnv3_b16,upcnv4_b16,icnv3_b16
python3 - <<'PY'
import re
p='scripts/conv_micro.py'; s=open(p).read()
if '"cnv5b_b16"' not in s:
    s=s.replace('    ("icnv5_b16", 16, 12, 16, 512, 256, 3, 1),','    ("icnv5_b16", 16, 12, 16, 512, 256, 3, 1),\n    ("cnv5b_b16", 16, 6, 8, 512, 512, 3, 1),\n    ("upcnv4_b16", 16, 24, 32, 128, 256, 3, 2),')
    open(p,'w').write(s)
PY
for v in 0 1; do
  echo "== TDE_BWD2_PF2=$v" >> $out
  TDE_BWD2_PF2=$v timeout -k 10 200 python -u scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad,wgrad --reps 20 --shapes $SH >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "^\.\|passed\|amdgpu.ids" $out
n=0
for v in 0 1 0 1; do
  n=$((n+1))
  TDE_BWD2_PF2=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/bench_${tag}_pf${v}_$n.json 2> gpurun_out/bench_${tag}_pf${v}_$n.err || { tail -20 gpurun_out/bench_${tag}_pf${v}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" gpurun_out/bench_${tag}_pf${v}_$n.json "pf2=$v"
done
