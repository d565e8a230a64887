set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv2d" > gpurun_out/s5_hwg_tests.log 2>&1; rc=$?; tail -4 gpurun_out/s5_hwg_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do echo "TDE_HWG=$v"; TDE_HWG=$v timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b,icnv1,icnv2 --reps 20 2>&1 | grep -v "amdgpu.ids\|== math" || exit 1; done
for b in 384 1536; do echo "TDE_HWG_BLOCKS=$b"; TDE_HWG_BLOCKS=$b timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b,icnv1,icnv2 --reps 20 2>&1 | grep -v "amdgpu.ids\|== math" || exit 1; done
