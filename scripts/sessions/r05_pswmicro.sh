set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
S=upcnv1_b16,upcnv2_b16,upcnv3_b16,cnv1p_b16,cnv2_b16,cnv3_b16,cnv4_b16,expup1_b16
for v in 8192 0; do
echo "== TDE_PSW_MINM=$v"
TDE_PSW_MINM=$v timeout -k 10 200 python3 scripts/conv_micro.py --math fp16x3 --shapes $S --modes wgrad,dgrad --reps 30 2>&1 | grep -v amdgpu.ids
done
