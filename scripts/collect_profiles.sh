#!/bin/bash
# Copy a round's judged evidence from gpurun_out/ into profiles/ (tracked).
set -eu
cd "$(dirname "$0")/.."
TAG=${1:-r01}
mkdir -p profiles
for w in config2 config3 config4 config5; do
  [ -f gpurun_out/bench_${TAG}_$w.json ] && cp gpurun_out/bench_${TAG}_$w.json profiles/bench_${TAG}_$w.json
done
cp gpurun_out/prof_${TAG}_config2/run_kernel_stats.csv profiles/${TAG}_config2_kernel_stats.csv
cp gpurun_out/kstats_${TAG}_config2.txt profiles/${TAG}_config2_kernel_stats_per_step.txt
cp gpurun_out/pmc_config2_fp32_b8.json profiles/pmc_config2_fp32_b8.json
ls -la profiles
