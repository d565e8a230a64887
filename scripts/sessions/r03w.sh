#!/bin/bash
# Round-3 validation of the current tree: the full GPU suite + smoke(), then the default bench line (config 4,
# secondary configs, CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=r03w bash scripts/sessions/r03_tests.sh
rc=$?; echo "[r03w] tests+smoke rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r03w.json 2> gpurun_out/bench_r03w.err
rc2=$?; echo "[r03w] bench rc=$rc2"; cat gpurun_out/bench_r03w.json | head -c 600; echo
exit $rc
