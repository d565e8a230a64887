set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
TDE_RING=8 $B > gpurun_out/bench_r05o_deep.json 2> gpurun_out/bench_r05o_deep.err || exit $?
TDE_RING=0 $B > gpurun_out/bench_r05o_off.json 2> gpurun_out/bench_r05o_off.err || exit $?
TDE_RING=8 $B > gpurun_out/bench_r05o_deep2.json 2> gpurun_out/bench_r05o_deep2.err || exit $?
TDE_RING=0 $B > gpurun_out/bench_r05o_off2.json 2> gpurun_out/bench_r05o_off2.err || exit $?
