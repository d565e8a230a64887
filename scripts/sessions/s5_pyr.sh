set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_nets.py tests/test_gpu_trainers.py tests/test_gpu_utils_lr.py > gpurun_out/s5_pyr_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s5_pyr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_pyr" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_pyr.log 2>&1 || exit $?
grep -h "depth_pyramid" $(find gpurun_out/prof_pyr -name '*kernel_stats.csv') | cut -d, -f1-4
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])"
