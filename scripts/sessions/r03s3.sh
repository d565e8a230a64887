#!/bin/bash
# Round-3 (session 3) re-check after the container was re-created and libtde.so rebuilt from the
# committed sources: full GPU suite + smoke(), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03s3 bash scripts/sessions/r03_tests.sh
rc=$?; echo "[r03s3] tests+smoke rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r03s3.json 2> gpurun_out/bench_r03s3.err
rc2=$?; echo "[r03s3] bench rc=$rc2"; head -c 600 gpurun_out/bench_r03s3.json; echo; [ $rc2 -ne 0 ] && exit $rc2
exit $rc
