#!/bin/bash
# Round 4: split-K slabs summed inside the small-M BatchNorm launch -- BN / conv kernel tests, trainer and
# full-size tests, then the default bench twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "bn or conv" --timeout 300 --timeout-method thread > gpurun_out/tests_r04u_k.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r04u_k.log; echo "[r04u] kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04u_t.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r04u_t.log; echo "[r04u] trainer tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/bench_r04u_$rep.json 2> gpurun_out/bench_r04u_$rep.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04u_$rep.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r04u_$rep.json'));print('default', d['value'], d['ms_per_step'])"
done
