#!/bin/bash
# Round 4, last: the whole GPU suite, smoke() and the default bench line on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04zz.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r04zz.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r04zz.json 2> gpurun_out/bench_r04zz.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04zz.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04zz.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['achieved'], {k: v['value'] for k, v in d['secondary'].items()})"
