set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/s5_wgrad_ab.txt
: > $OUT
run() { echo "== $*" >> $OUT; env "$@" timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b,icnv1,icnv2,cnv2b,icnv3 --reps 20 2>&1 | grep -v "amdgpu.ids\|== math" >> $OUT || exit 1; }
run TDE_SPLIT_TARGET=512
run TDE_SPLIT_TARGET=1024
run TDE_SPLIT_TARGET=2048
run TDE_SPLIT_TARGET=4096
run TDE_MATH3_WGRAD_MIN_BN=16
run TDE_MATH3_WGRAD_MIN_BN=16 TDE_SPLIT_TARGET=2048
run TDE_NARROW_MATH=2 TDE_MATH3_WGRAD_MIN_BN=16
run TDE_SPLIT_MINKT=16
cat $OUT
