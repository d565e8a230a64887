set -u
cd $GRAFT_REPO_ROOT
for v in 0 1 2 3; do echo "TDE_HWG_DIAG=$v"; TDE_HWG_DIAG=$v timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b,icnv1,icnv2 --reps 20 2>&1 | grep -v "amdgpu.ids\|== math" || exit 1; done
