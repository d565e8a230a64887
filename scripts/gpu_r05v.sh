set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
TDE_C4_SPLIT=1 $B > gpurun_out/bench_r05v_split.json 2> gpurun_out/bench_r05v_split.err || exit $?
$B > gpurun_out/bench_r05v_base.json 2> gpurun_out/bench_r05v_base.err || exit $?
TDE_C4_SPLIT=1 $B > gpurun_out/bench_r05v_split2.json 2> gpurun_out/bench_r05v_split2.err || exit $?
$B > gpurun_out/bench_r05v_base2.json 2> gpurun_out/bench_r05v_base2.err || exit $?
TDE_C4_SPLIT=1 timeout -k 10 300 python -u probe/step_timeline.py gpurun_out/timeline_r05v_split.txt > gpurun_out/timeline_r05v_split.log 2>&1
