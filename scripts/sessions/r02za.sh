#!/bin/bash
# Pre-split halo weights (one tde_conv2d_split_weights launch per forward): full GPU suite, smoke, benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r02za
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
for WL in config2 config4 config2 config4; do
  timeout -k 10 200 python -u bench.py --workload $WL --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_$WL.json 2>gpurun_out/${TAG}_$WL.err || { tail -5 gpurun_out/${TAG}_$WL.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$WL.json'));print('$WL',d['value'],d['ms_per_step'])"
done
timeout -k 10 300 python -u scripts/loader_bench.py --shape config2 > gpurun_out/${TAG}_loader_config2.json 2> gpurun_out/${TAG}_loader.err || { tail -5 gpurun_out/${TAG}_loader.err; exit 1; }
cat gpurun_out/${TAG}_loader_config2.json
