#!/bin/bash
# Is the config-4 two-stream overlap real?  Graph-concurrency probe, then bench with the net overlap on / off,
# graph / eager, and an eager kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u probe/graph_concurrency.py > gpurun_out/r03r_graphconc.log 2>&1
rc=$?; echo "[r03r] probe rc=$rc"; grep "\[graph_conc" gpurun_out/r03r_graphconc.log; [ $rc -ne 0 ] && exit $rc
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-secondary "$@" \
    > gpurun_out/ab_r03r_$tag.json 2> gpurun_out/ab_r03r_$tag.err
  local rc=$?
  echo "[r03r] $tag rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03r_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
run graph_ov || exit 1
run graph_noov --net-overlap off || exit 1
run eager_ov --no-graph || exit 1
run eager_noov --no-graph --net-overlap off || exit 1
run graph_ov_nowg --wgrad-overlap off || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/prof_r03r_eager" -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-graph > gpurun_out/prof_r03r_eager.log 2>&1
rc=$?; echo "[r03r] eager trace rc=$rc"
