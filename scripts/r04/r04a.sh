#!/bin/bash
# Round-4 re-entry: default bench line + per-layer HIP-event profile of configs 4 and 2 (fp16x3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err
rc=$?; echo "[r04a] bench rc=$rc"; head -c 400 gpurun_out/bench_r04a.json; echo; [ $rc -ne 0 ] && exit $rc
for w in config4 config2; do
  timeout -k 10 300 python scripts/layer_profile.py --workload $w --math fp16x3 --top 200 --loss-vs 833 \
    > gpurun_out/layers_r04a_$w.txt 2> gpurun_out/layers_r04a_$w.err
  rc=$?; echo "[r04a] layers $w rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
