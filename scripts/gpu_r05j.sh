set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T tests/test_gpu_kernels.py > gpurun_out/tests_r05j.log 2>&1 || exit $?
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
$B > gpurun_out/bench_r05j_new.json 2> gpurun_out/bench_r05j_new.err || exit $?
TDE_HEAD_RWK=0 $B > gpurun_out/bench_r05j_norwk.json 2> gpurun_out/bench_r05j_norwk.err || exit $?
$B --exchange on > gpurun_out/bench_r05j_xon.json 2> gpurun_out/bench_r05j_xon.err || exit $?
$B > gpurun_out/bench_r05j_new2.json 2> gpurun_out/bench_r05j_new2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05j -o run --output-format csv -- python3 scripts/layer_profile.py --workload config4 --math fp16x3 --top 5 > gpurun_out/prof_r05j.log 2>&1
