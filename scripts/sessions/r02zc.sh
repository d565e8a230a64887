#!/bin/bash
# Round-2 kernel-trace profiles of the current tree (rocprofv3 --kernel-trace --stats): config 2 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02zc}
for WL in ${WLS:-config2 config4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_$WL" -o run --output-format csv \
    -- python3 bench.py --workload "$WL" --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/prof_${TAG}_$WL.log 2>&1 || { echo "rocprofv3 $WL failed"; exit 1; }
  tail -1 gpurun_out/prof_${TAG}_$WL.log | cut -c1-160
done
