set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_launch_status.py > gpurun_out/tests_r05f_kernels.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline > gpurun_out/bench_r05f_ring.json 2> gpurun_out/bench_r05f_ring.err || exit $?
TDE_RING=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline > gpurun_out/bench_r05f_noring.json 2> gpurun_out/bench_r05f_noring.err || exit $?
TDE_RING_WGRAD=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline > gpurun_out/bench_r05f_nowg.json 2> gpurun_out/bench_r05f_nowg.err || exit $?
timeout -k 10 300 python -u scripts/layer_profile.py --workload config4 --math fp16x3 --top 150 --loss-vs 400 > gpurun_out/layers_r05f_ring.txt 2>&1 || exit $?
TDE_RING=0 timeout -k 10 300 python -u scripts/layer_profile.py --workload config4 --math fp16x3 --top 150 --loss-vs 400 > gpurun_out/layers_r05f_noring.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py tests/test_gpu_trainers.py tests/test_gpu_nets.py > gpurun_out/tests_r05f_train.log 2>&1
