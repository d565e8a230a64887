#!/bin/bash
# Loader with JPEG decode in worker processes (shared-memory staging): loader GPU tests, then the loader
# measurements with 16 processes vs 16 threads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dataloader.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02zf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02zf_tests.log
[ $rc -eq 0 ] || exit $rc
for p in 16 0; do
  timeout -k 10 300 python -u scripts/loader_bench.py --shape config2 --procs $p > gpurun_out/r02zf_loader_p$p.json 2>> gpurun_out/r02zf_loader.err || { tail -5 gpurun_out/r02zf_loader.err; exit 1; }
  cat gpurun_out/r02zf_loader_p$p.json
done
timeout -k 10 300 python -u scripts/loader_bench.py --shape ref --batches 20 --procs 16 > gpurun_out/r02zf_loader_ref.json 2>> gpurun_out/r02zf_loader.err || { tail -5 gpurun_out/r02zf_loader.err; exit 1; }
cat gpurun_out/r02zf_loader_ref.json
ls /dev/shm | head -5
