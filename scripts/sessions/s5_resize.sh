set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_nets.py -k "resize or bilinear or disp_net or config2" > gpurun_out/s5_resize_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s5_resize_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/layer_profile.py --math bf16x6r --top 300 2>&1 | grep -E "resize|total"
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])"
