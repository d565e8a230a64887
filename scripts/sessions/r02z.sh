#!/bin/bash
# Pipelined loader + exact-x2 bilinear kernels: GPU tests (loader, kernels, nets, trainers), loader measurements,
# config-2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_dataloader.py tests/test_gpu_kernels.py tests/test_gpu_nets.py tests/test_gpu_trainers.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02z_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02z_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/loader_bench.py --shape config2 > gpurun_out/r02z_loader_config2.json 2> gpurun_out/r02z_loader.err || { tail -5 gpurun_out/r02z_loader.err; exit 1; }
cat gpurun_out/r02z_loader_config2.json
timeout -k 10 300 python -u scripts/loader_bench.py --shape ref --batches 20 > gpurun_out/r02z_loader_ref.json 2>> gpurun_out/r02z_loader.err || { tail -5 gpurun_out/r02z_loader.err; exit 1; }
cat gpurun_out/r02z_loader_ref.json
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r02z_b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02z_b.json'));print('config2',d['value'],d['ms_per_step'],d['kernel_breakdown_ms']['resize'])"
done
