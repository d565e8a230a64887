set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread"
$T tests/test_gpu_kernels.py -k "head" > gpurun_out/tests_r05m_heads.log 2>&1 || exit $?
$T tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_nets.py > gpurun_out/tests_r05m.log 2>&1 || exit $?
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
$B > gpurun_out/bench_r05m_off.json 2> gpurun_out/bench_r05m_off.err || exit $?
$B --exchange on --exchange-mode inline > gpurun_out/bench_r05m_inl32.json 2> gpurun_out/bench_r05m_inl32.err || exit $?
$B --exchange on --exchange-mode inline --bucket-mb 256 > gpurun_out/bench_r05m_inl256.json 2> gpurun_out/bench_r05m_inl256.err || exit $?
$B --exchange on --bucket-mb 256 > gpurun_out/bench_r05m_g256.json 2> gpurun_out/bench_r05m_g256.err || exit $?
$B > gpurun_out/bench_r05m_off2.json 2> gpurun_out/bench_r05m_off2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05m -o run --output-format csv -- python3 scripts/layer_profile.py --workload config4 --math fp16x3 --top 5 > gpurun_out/prof_r05m.log 2>&1
