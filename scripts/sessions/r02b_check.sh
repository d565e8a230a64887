#!/bin/bash
# Round-2 re-entry check on a fresh box: full GPU parity suite, smoke, default bench, kernel-trace profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02b_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r02b_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02b_smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/r02b_smoke.log
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 300 python -u bench.py > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err
rc3=$?; echo "bench rc=$rc3"; cat gpurun_out/r02b_bench.json
[ $rc3 -eq 0 ] || exit $rc3
bash scripts/sessions/r02_prof.sh r02b > /dev/null 2>&1
echo "prof rc=$?"; head -40 gpurun_out/kstats_r02b.txt
exit $rc
