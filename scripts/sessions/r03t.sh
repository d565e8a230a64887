#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u probe/graph_concurrency.py > gpurun_out/r03t_gc.log 2>&1
rc=$?; echo "[r03t] rc=$rc"; grep "\[graph_conc" gpurun_out/r03t_gc.log; tail -3 gpurun_out/r03t_gc.log
