#!/bin/bash
# Round evidence in one GPU session: every workload's bench line, the rocprofv3 kernel-trace summary of
# the default bench command, and the PMC HBM traffic of the headline workload.  Outputs land in
# gpurun_out/; copy the ones to be judged into profiles/ (scripts/collect_profiles.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
bash scripts/pmc.sh "$TAG" config2 fp32 8 || exit $?
cp gpurun_out/pmc_config2_fp32_b8.json profiles/ 2>/dev/null
STEPS=${STEPS:-100} bash scripts/bench_all.sh "$TAG" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_config2" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}_config2.log 2>&1
rc=$?; echo "[round_profile] rocprofv3 rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/kstats.py gpurun_out/prof_${TAG}_config2/run_kernel_stats.csv 29 30 > gpurun_out/kstats_${TAG}_config2.txt
head -12 gpurun_out/kstats_${TAG}_config2.txt
