set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > gpurun_out/t_kern.log 2>&1; rc=$?; tail -3 gpurun_out/t_kern.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nets.py tests/test_golden.py tests/test_gpu_utils_lr.py > gpurun_out/t_nets.log 2>&1; rc=$?; tail -3 gpurun_out/t_nets.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/conv_micro.py --math all --reps 20 > gpurun_out/micro.log 2>&1 || exit $?
cat gpurun_out/micro.log
for m in fp32 bf16x6 bf16x6r bf16x3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --math $m > gpurun_out/bench_$m.json 2>gpurun_out/bench_$m.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_$m.json'));print('$m',d['ms_per_step'],d['value'],d['roofline']['conv_ms_per_step'])"
done
