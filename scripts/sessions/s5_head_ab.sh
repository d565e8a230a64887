set -u
cd $GRAFT_REPO_ROOT
for v in "TDE_HEAD_PPL=8" "TDE_HEAD_PPL=2" "TDE_HEAD_PPL=4" "TDE_HEAD_PPL=2 TDE_HEAD_BLOCKS=4096"; do echo "$v"; env $v timeout -k 10 120 python scripts/layer_profile.py --math bf16x6r --top 200 2>&1 | grep -E "head_|total" || exit 1; done
