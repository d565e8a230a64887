set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
TDE_RING=0 $B > gpurun_out/bench_r05g_noring.json 2> gpurun_out/bench_r05g_noring.err || exit $?
$B > gpurun_out/bench_r05g_ring.json 2> gpurun_out/bench_r05g_ring.err || exit $?
TDE_RING_WGRAD=0 $B > gpurun_out/bench_r05g_nowg.json 2> gpurun_out/bench_r05g_nowg.err || exit $?
TDE_SPLIT_HEAD=3 $B > gpurun_out/bench_r05g_split3.json 2> gpurun_out/bench_r05g_split3.err || exit $?
TDE_RING=0 $B > gpurun_out/bench_r05g_noring2.json 2> gpurun_out/bench_r05g_noring2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05g_ring -o run --output-format csv -- python3 scripts/layer_profile.py --workload config4 --math fp16x3 --top 5 > gpurun_out/prof_r05g_ring.log 2>&1 || exit $?
TDE_RING=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05g_noring -o run --output-format csv -- python3 scripts/layer_profile.py --workload config4 --math fp16x3 --top 5 > gpurun_out/prof_r05g_noring.log 2>&1
