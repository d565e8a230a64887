set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/s4_gpu_tests.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/s4_gpu_tests.log | tail -3; grep FAILED gpurun_out/s4_gpu_tests.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4_smoke.log 2>&1 || exit $?
cat gpurun_out/s4_smoke.log
for m in fp32 bf16x6r; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 20 --math $m > gpurun_out/s4_bench_$m.json 2>gpurun_out/s4_bench_$m.err || exit $?
  cat gpurun_out/s4_bench_$m.json
done
