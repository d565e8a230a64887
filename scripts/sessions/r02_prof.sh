#!/bin/bash
# Kernel-trace summary + per-layer table of the default config-2 step (diagnostic, round 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02a}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}" -o run --output-format csv \
  -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py "$(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1)" 124 60 > gpurun_out/kstats_${TAG}.txt
cat gpurun_out/kstats_${TAG}.txt
timeout -k 10 200 python3 scripts/layer_profile.py --math fp16x3 --top 90 > gpurun_out/layers_${TAG}.txt 2>&1
rc=$?; echo "layers rc=$rc"; cat gpurun_out/layers_${TAG}.txt
