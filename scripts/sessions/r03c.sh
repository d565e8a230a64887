#!/bin/bash
# Round 3: new-feature GPU tests (new nets, deterministic scatter, full-size parity), then the profiling
# session (scripts/sessions/r03a.sh).  A test assertion failure does not stop the profiling; a crash / timeout does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_nets.py tests/test_gpu_kernels.py tests/test_gpu_trainers.py \
  tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread \
  -k "sfm or bn_free or bias_relu or head_fwd_bwd or resize_fwd_bwd or trainers or fullsize" > gpurun_out/r03c_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r03c_tests.log
case $rc in 0|1) ;; *) echo "[r03c] tests rc=$rc: stopping"; exit $rc;; esac
bash scripts/sessions/r03a.sh
