#!/bin/bash
# Round 4: SyncBN tests (world-1 capture, world-2 gloo config-4 grouped SyncBN), then planner-knob A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py \
  tests/test_gpu_ddp_world2.py > gpurun_out/tests_r04h.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/tests_r04h.log | tail -20; echo "[r04h] tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
TAG=r04f bash scripts/r04/ab_env.sh base TDE_DECONV_PS_MINBLOCKS=192 TDE_BM64_MAXM=16384 TDE_SPLIT_MINKT=6
exit $rc
