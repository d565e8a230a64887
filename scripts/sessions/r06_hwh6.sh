# Round 6: halo filter gradient after the staging-index hoist -- tests, per-layer times, SQ counters.
# Usage: r06_hwh6.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06o}
out=gpurun_out/hwh6_${tag}.txt
: > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread \
  -k "halo or fp16x3_operand_bounds or conv2d_fwd_bwd" >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -2 $out
timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes wgrad --reps 30 \
  --shapes cnv1b_b16,icnv1_b16,icnv2_b16,cnv1p_b16,upcnv1_b16,expup1_b16 >> $out 2>&1 || { tail -20 $out; exit 1; }
grep -v "^\.\|passed\|amdgpu.ids" $out
bash scripts/sessions/r06_hwh_pmc.sh $tag
