set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T tests/test_gpu_kernels.py -k "ring or pixel or presplit" > gpurun_out/tests_r05h.log 2>&1 || exit $?
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
$B > gpurun_out/bench_r05h_fwd.json 2> gpurun_out/bench_r05h_fwd.err || exit $?
TDE_RING=0 $B > gpurun_out/bench_r05h_noring.json 2> gpurun_out/bench_r05h_noring.err || exit $?
$B > gpurun_out/bench_r05h_fwd2.json 2> gpurun_out/bench_r05h_fwd2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05h_fwd -o run --output-format csv -- python3 scripts/layer_profile.py --workload config4 --math fp16x3 --top 5 > gpurun_out/prof_r05h_fwd.log 2>&1
