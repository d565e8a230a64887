set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv2d" > gpurun_out/s5_hwg2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s5_hwg2_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "TDE_HWG=0" "TDE_HWG_MIN_ITEMS=1" "TDE_HWG_MIN_ITEMS=1 TDE_HWG_DIAG=1" "TDE_HWG_MIN_ITEMS=1 TDE_HWG_DIAG=2"; do echo "$v"; env $v timeout -k 10 120 python scripts/conv_micro.py --math bf16x6r --modes wgrad --shapes cnv1b,icnv1,icnv2 --reps 20 2>&1 | grep -v "amdgpu.ids\|== math" || exit 1; done
