#!/bin/bash
# Loader-fed training: 16 decode processes vs 16 threads, default and 0.2 ms GIL switch interval.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 16 0; do
  timeout -k 10 300 python -u scripts/loader_bench.py --shape config2 --procs $p > gpurun_out/r02zg_loader_p$p.json 2>> gpurun_out/r02zg_loader.err || { tail -5 gpurun_out/r02zg_loader.err; exit 1; }
  cat gpurun_out/r02zg_loader_p$p.json
done
