set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T tests/test_gpu_ddp.py > gpurun_out/tests_r05l.log 2>&1 || exit $?
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
$B --exchange on --exchange-mode inline > gpurun_out/bench_r05l_inl32.json 2> gpurun_out/bench_r05l_inl32.err || exit $?
$B --exchange on --exchange-mode inline --bucket-mb 256 > gpurun_out/bench_r05l_inl256.json 2> gpurun_out/bench_r05l_inl256.err || exit $?
$B > gpurun_out/bench_r05l_off.json 2> gpurun_out/bench_r05l_off.err || exit $?
$B --exchange on --bucket-mb 256 > gpurun_out/bench_r05l_g256.json 2> gpurun_out/bench_r05l_g256.err || exit $?
$B --exchange on --exchange-mode inline --bucket-mb 256 > gpurun_out/bench_r05l_inl256b.json 2> gpurun_out/bench_r05l_inl256b.err || exit $?
