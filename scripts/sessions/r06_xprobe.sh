# Round 6: why the segments-mode exchange costs ~28 % at world 1 (bench_r06c_xseg_*): host cost of the eager
# all-reduce (ProcessGroupNCCL vs direct RCCL), the graph-mode exchange after the one-level fork change, and a
# kernel trace of the segments-mode bench.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 probe/exchange_host.py > gpurun_out/r06_xhost.txt 2>&1 || { tail -5 gpurun_out/r06_xhost.txt; exit 1; }
tail -1 gpurun_out/r06_xhost.txt
timeout -k 10 300 python3 bench.py --exchange on --exchange-mode graph --no-cpu-baseline --no-secondary --steps 60 --warmup 15 > gpurun_out/bench_r06d_xgraph.json 2> gpurun_out/bench_r06d_xgraph.err || { tail -5 gpurun_out/bench_r06d_xgraph.err; exit 1; }
head -c 250 gpurun_out/bench_r06d_xgraph.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r06d_xseg" -o run --output-format csv -- python3 bench.py --exchange on --no-cpu-baseline --no-secondary --steps 30 --warmup 10 > gpurun_out/prof_r06d_xseg.log 2>&1 || { tail -5 gpurun_out/prof_r06d_xseg.log; exit 1; }
echo done
