#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u probe/cu_mask.py > gpurun_out/r03u_cumask.log 2>&1
rc=$?; echo "[r03u] rc=$rc"; grep "\[cu_mask" gpurun_out/r03u_cumask.log; tail -3 gpurun_out/r03u_cumask.log
