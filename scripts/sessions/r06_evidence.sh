# Round 6: GPU suite (-x, one process, as the driver), smoke, the default bench line, the exchange A/B at world 1
# (segments mode with 256 / 64 MB buckets) and the rocprofv3 kernel-trace summary of the default bench.
# Every GPU step under its own time limit; the script stops at the first failing step.  Usage: r06_evidence.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06}
timeout -k 10 900 python -u -m pytest tests -x -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_${tag}.txt 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_${tag}.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${tag}.txt 2>&1 || { tail -5 gpurun_out/smoke_${tag}.txt; exit 1; }
timeout -k 10 500 python3 bench.py --graph-spans gpurun_out/spans_${tag}.json > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || { tail -5 gpurun_out/bench_${tag}.err; exit 1; }
cat gpurun_out/bench_${tag}.json | head -c 600; echo
timeout -k 10 300 python3 scripts/infer_bench.py --iters 100 > gpurun_out/infer_${tag}.json 2> gpurun_out/infer_${tag}.err || { tail -5 gpurun_out/infer_${tag}.err; exit 1; }
for b in 256; do
  timeout -k 10 300 python3 bench.py --exchange on --bucket-mb $b --no-cpu-baseline --no-secondary --steps 60 --warmup 15 > gpurun_out/bench_${tag}_xseg_b$b.json 2> gpurun_out/bench_${tag}_xseg_b$b.err || { tail -5 gpurun_out/bench_${tag}_xseg_b$b.err; exit 1; }
  head -c 300 gpurun_out/bench_${tag}_xseg_b$b.json; echo
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${tag}" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 100 --warmup 20 > gpurun_out/prof_${tag}.log 2>&1 || { tail -5 gpurun_out/prof_${tag}.log; exit 1; }
echo done
