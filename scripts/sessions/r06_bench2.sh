# Round 6: GPU kernel/fullsize tests touching the conv kernels, then two default bench runs.  Usage: r06_bench2.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06q}
out=gpurun_out/tests_${tag}.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_nets.py -x -q \
  --timeout 150 --timeout-method thread > $out 2>&1 || { tail -30 $out; exit 1; }
tail -2 $out
for n in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/bench_${tag}_$n.json 2> gpurun_out/bench_${tag}_$n.err || { tail -20 gpurun_out/bench_${tag}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" gpurun_out/bench_${tag}_$n.json
done
