#!/bin/bash
# Round 4: row-walk 3x3 heads -- head kernel tests, full-size parity, then config 4 / config 2 A/B against the
# halo-tiled head kernels (TDE_HEAD_RW=0), alternating x2 on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_fullsize.py tests/test_gpu_nets.py -k "head or fullsize or full or config" > gpurun_out/tests_r04j.log 2>&1
rc=$?; tail -4 gpurun_out/tests_r04j.log; echo "[r04j] tests rc=$rc"
case $rc in 0) ;; *) grep -E "^(FAILED|E )" gpurun_out/tests_r04j.log | head -20; exit $rc;; esac
TAG=r04j bash scripts/r04/ab_env.sh base TDE_HEAD_RW=0
