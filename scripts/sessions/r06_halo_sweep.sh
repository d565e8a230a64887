# Round 6: halo conv plan sweep (TDE_HALO_NW x TDE_HALO_TN x TDE_HALO_MINCH) on the config-4 halo layers; each plan
# printed by TDE_HALO_VERBOSE.  Usage: r06_halo_sweep.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06x}
out=gpurun_out/halosweep_${tag}.txt
: > $out
SH=cnv1b_b16,icnv1_b16,icnv2_b16,cnv2b_b16,icnv3_b16
echo "== default" >> $out
TDE_HALO_VERBOSE=1 timeout -k 10 100 python -u scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad --reps 20 --shapes $SH >> $out 2>&1 || exit 1
for nw in 4 8; do for tn in 1 2 4; do for mc in 1 2; do
  echo "== NW $nw TN $tn MINCH $mc" >> $out
  TDE_HALO_VERBOSE=1 TDE_HALO_NW=$nw TDE_HALO_TN=$tn TDE_HALO_MINCH=$mc timeout -k 10 100 python -u scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad --reps 20 --shapes $SH >> $out 2>&1 || { echo "fail nw $nw tn $tn mc $mc" >> $out; }
done; done; done
grep -c "==" $out
