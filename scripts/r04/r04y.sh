#!/bin/bash
# Round 4: final-binary sanity check (the library rebuilt after the A/B build flags were added; defaults unchanged):
# BN / conv kernel tests, DDP suites, smoke and the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ddp.py tests/test_gpu_ddp_world2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04y.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r04y.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-secondary > gpurun_out/bench_r04y.json 2> gpurun_out/bench_r04y.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04y.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04y.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['traffic'])"
