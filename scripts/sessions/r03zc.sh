#!/bin/bash
# Config 4 as one linear graph (no net overlap, no filter-gradient side streams) and with only depth_net's
# filter-gradient branch, against the default pieces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary "$@" \
    > gpurun_out/ab_r03zc_$tag.json 2> gpurun_out/ab_r03zc_$tag.err
  local rc=$?
  echo "[r03zc] $tag rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03zc_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
for r in 1 2; do
  run default$r || exit 1
  run linear$r --net-overlap off --wgrad-overlap off || exit 1
  run onegraph_wgpair$r --net-overlap off --wgrad-progs pair || exit 1
done
echo "[r03zc] done"
