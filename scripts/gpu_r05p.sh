set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10 1100 python -u -m pytest -x -q --timeout 900 --timeout-method thread"
$T tests/test_gpu_trainers.py tests/test_gpu_kernels.py tests/test_gpu_launch_status.py tests/test_gpu_nets.py tests/test_gpu_inference.py tests/test_gpu_checkpoint.py tests/test_gpu_dataloader.py tests/test_gpu_sig_loss.py tests/test_gpu_utils_lr.py tests/test_gpu_ddp.py tests/test_gpu_ddp_world2.py > gpurun_out/tests_r05p.log 2>&1
