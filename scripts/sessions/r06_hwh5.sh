# Round 6: halo filter-gradient grid size sweep (TDE_HWG_BLOCKS) on the config-4 shapes.  Usage: r06_hwh5.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06m}
out=gpurun_out/hwh5_${tag}.txt
: > $out
for nb in 768 256 512 1024 1536 2304; do
  echo "== TDE_HWG_BLOCKS=$nb" >> $out
  TDE_HWG_BLOCKS=$nb timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes wgrad --reps 30 \
    --shapes cnv1b_b16,icnv1_b16,icnv2_b16,cnv1p_b16,upcnv1_b16,expup1_b16 >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "amdgpu.ids" $out
