set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
for k in 0 1 2 3; do
TDE_STREAM_PAD=$k $B > gpurun_out/bench_r05u_pad$k.json 2> gpurun_out/bench_r05u_pad$k.err || exit $?
done
