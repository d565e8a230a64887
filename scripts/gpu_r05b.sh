set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline --graph-spans gpurun_out/spans_r05b.json > gpurun_out/bench_r05b.json 2> gpurun_out/bench_r05b.err || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_launch_status.py tests/test_gpu_fullsize.py -k "launch_status or benched" > gpurun_out/tests_r05b.log 2>&1
