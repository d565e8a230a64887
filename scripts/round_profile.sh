#!/bin/bash
# Round evidence in one GPU session: the default bench line (config 2, with CPU baseline and depth L1 vs
# the reference restatement), the rocprofv3 kernel-trace summary of the same command, the PMC HBM
# traffic of the headline workload, a per-layer table, and the other workloads' bench lines.
# Outputs land in gpurun_out/; copy the judged ones into profiles/ (scripts/collect_profiles.sh TAG).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
MATH=${MATH:-bf16x6r}
stop() { echo "[round_profile] $1 rc=$2"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 400 python bench.py --steps 100 --warmup 20 --math "$MATH" > gpurun_out/bench_${TAG}_config2.json \
  2> gpurun_out/bench_${TAG}_config2.err
stop bench $?
cat gpurun_out/bench_${TAG}_config2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_config2" -o run --output-format csv \
  -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --math "$MATH" > gpurun_out/prof_${TAG}_config2.log 2>&1
stop rocprofv3 $?
# 2 eager steps + 2 capture-warmup steps + 20 warmup + 100 timed
python3 scripts/kstats.py "$(find gpurun_out/prof_${TAG}_config2 -name '*kernel_stats.csv' | head -1)" 124 40 \
  > gpurun_out/kstats_${TAG}_config2.txt
head -15 gpurun_out/kstats_${TAG}_config2.txt
bash scripts/pmc.sh "$TAG" config2 "$MATH" 8
stop pmc $?
timeout -k 10 200 python3 scripts/layer_profile.py --math "$MATH" --top 60 > gpurun_out/layers_${TAG}_config2.txt 2>&1
stop layer_profile $?
if [ "${ALL:-1}" = "1" ]; then
  for w in config3 config4 config5; do
    timeout -k 10 400 python bench.py --workload $w --steps 30 --warmup 5 --math "$MATH" \
      > gpurun_out/bench_${TAG}_$w.json 2> gpurun_out/bench_${TAG}_$w.err
    stop "bench $w" $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'], d.get('depth_l1_vs_ref',{}).get('worst_max_rel'))" gpurun_out/bench_${TAG}_$w.json $w
  done
fi
