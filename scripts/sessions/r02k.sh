#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "conv or deconv" --timeout 120 --timeout-method thread > gpurun_out/r02k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02k_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/conv_micro.py --math fp16x3 --reps 20 > gpurun_out/r02k_micro.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r02k_micro.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r02k_bench.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/r02k_bench.json'));print('bench',d['value'],d['ms_per_step'])"
MATH=fp16x3 bash scripts/conv_pmc.sh icnv5 fwd i5f2 | tail -20
