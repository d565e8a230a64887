set -u
cd $GRAFT_REPO_ROOT
for u in 2 4 8; do echo "unroll $u"; TDE_LIBRARY=$PWD/variants/libtde_u$u.so timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b --reps 30 2>&1 | grep -v "amdgpu.ids\|== math" || exit 1; done
echo "shipped (TP128, unroll 2, no pipelining)"; timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b --reps 30 2>&1 | grep -v "amdgpu.ids\|== math" || exit 1
TDE_LIBRARY=$PWD/variants/libtde_u2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv2d" 2>&1 | tail -1
