#!/bin/bash
# Re-entry check of the committed tree: full GPU suite + smoke(), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03s2a bash scripts/sessions/r03_tests.sh
rc=$?; echo "[r03s2a] tests+smoke rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r03s2a.json 2> gpurun_out/bench_r03s2a.err
rc2=$?; echo "[r03s2a] bench rc=$rc2"; head -c 300 gpurun_out/bench_r03s2a.json; echo
exit $(( rc ? rc : rc2 ))
