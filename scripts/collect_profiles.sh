#!/bin/bash
# Copy a round's judged evidence from gpurun_out/ into profiles/ (tracked).
set -eu
cd "$(dirname "$0")/.."
TAG=${1:-r01}
MATH=${MATH:-bf16x6r}
mkdir -p profiles
for w in config2 config3 config4 config5; do
  [ -f gpurun_out/bench_${TAG}_$w.json ] && cp gpurun_out/bench_${TAG}_$w.json profiles/bench_${TAG}_$w.json
done
f=$(find gpurun_out/prof_${TAG}_config2 -name '*kernel_stats.csv' | head -1)
cp "$f" profiles/${TAG}_config2_kernel_stats.csv
cp gpurun_out/kstats_${TAG}_config2.txt profiles/${TAG}_config2_kernel_stats_per_step.txt
cp gpurun_out/pmc_config2_${MATH}_b8.json profiles/pmc_config2_${MATH}_b8.json
[ -f gpurun_out/layers_${TAG}_config2.txt ] && cp gpurun_out/layers_${TAG}_config2.txt profiles/
ls -la profiles
