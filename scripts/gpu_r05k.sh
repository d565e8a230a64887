set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-secondary --no-cpu-baseline"
for mb in 64 128 256; do
$B --exchange on --bucket-mb $mb > gpurun_out/bench_r05k_xon_b$mb.json 2> gpurun_out/bench_r05k_xon_b$mb.err || exit $?
done
$B --exchange on --bucket-mb 512 > gpurun_out/bench_r05k_xon_b512b.json 2> gpurun_out/bench_r05k_xon_b512b.err || exit $?
$B > gpurun_out/bench_r05k_off2.json 2> gpurun_out/bench_r05k_off2.err || exit $?
