#!/bin/bash
# DDP / deterministic GPU tests, then the profiling session (bench config 4 + secondary + CPU leg, kernel
# trace, PMC passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_trainers.py -q --timeout 300 \
  --timeout-method thread -k "ddp or deterministic or exchange" > gpurun_out/r03f_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03f_tests.log
case $rc in 0|1) ;; *) echo "[r03f] tests rc=$rc: stopping"; exit $rc;; esac
TAG=r03f bash scripts/sessions/r03a.sh
