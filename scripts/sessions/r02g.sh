#!/bin/bash
# Full GPU suite on the staged-split build; bench; timing experiments (filter gradients skipped / unfused).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r02g_tests.log
[ $rc -le 1 ] || exit $rc
for envs in "X=0" "TDE_SKIP_WGRAD=1" "TDE_BWD_FUSE=0"; do
  env $envs timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r02g_bench.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02g_bench.json'));print('$envs',d['value'],d['ms_per_step'])"
done
