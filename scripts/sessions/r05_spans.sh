set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --graph-spans gpurun_out/spans_r05ps.json > gpurun_out/bench_r05ps.json 2> gpurun_out/bench_r05ps.err || { tail -5 gpurun_out/bench_r05ps.err; exit 1; }
python3 scripts/spans_table.py gpurun_out/spans_r05ps.json 70 > gpurun_out/spans_r05ps.txt
tail -8 gpurun_out/spans_r05ps.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r05ps" -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/prof_r05ps.log 2>&1 || { tail -5 gpurun_out/prof_r05ps.log; exit 1; }
find gpurun_out/prof_r05ps -name '*kernel_stats.csv'
