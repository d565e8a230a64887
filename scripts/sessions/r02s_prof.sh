#!/bin/bash
# Kernel-trace profiles of the given workloads (round 2, session 4): rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02s}
for WL in ${WLS:-config4 config3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_$WL" -o run --output-format csv \
    -- python3 bench.py --workload "$WL" --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/prof_${TAG}_$WL.log 2>&1 || { echo "rocprofv3 $WL failed rc=$?"; exit 1; }
  tail -1 gpurun_out/prof_${TAG}_$WL.log | cut -c1-200
done
