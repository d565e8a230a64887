#!/bin/bash
# Input pipeline (imageselect_Dataloader_optflow): GPU tests, then loader / kernel / fed-training measurements.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dataloader.py tests/test_abi.py -x -q -m "gpu or not gpu" --timeout 120 --timeout-method thread > gpurun_out/r02y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02y_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/loader_bench.py --shape config2 > gpurun_out/r02y_loader_config2.json 2> gpurun_out/r02y_loader.err || { tail -5 gpurun_out/r02y_loader.err; exit 1; }
cat gpurun_out/r02y_loader_config2.json
timeout -k 10 300 python -u scripts/loader_bench.py --shape ref --batches 20 > gpurun_out/r02y_loader_ref.json 2>> gpurun_out/r02y_loader.err || { tail -5 gpurun_out/r02y_loader.err; exit 1; }
cat gpurun_out/r02y_loader_ref.json
