#!/bin/bash
# Full GPU test suite + smoke() (one process for the tests), output under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/tests_${TAG}.log 2>&1
rc=$?; tail -25 gpurun_out/tests_${TAG}.log
case $rc in 0|1) ;; *) echo "[tests] rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc2=$?; tail -2 gpurun_out/smoke_${TAG}.log
[ $rc -ne 0 ] && exit $rc
exit $rc2
