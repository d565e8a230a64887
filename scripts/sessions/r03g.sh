#!/bin/bash
# A/B: HW queue count and single-graph capture for the config-4 step; the repeated single-graph capture probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
    > gpurun_out/ab_r03g_$tag.json 2> gpurun_out/ab_r03g_$tag.err
  local rc=$?
  echo "[r03g] $tag rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r03g_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
run base TDE_X=0 || exit 1
run q8 GPU_MAX_HW_QUEUES=8 || exit 1
run single TDE_C4_SINGLE_GRAPH=1 || exit 1
run q8single GPU_MAX_HW_QUEUES=8 TDE_C4_SINGLE_GRAPH=1 || exit 1
run noinline TDE_C4_INLINE_ADAM=0 || exit 1
run q8b GPU_MAX_HW_QUEUES=8 || exit 1
timeout -k 10 300 python -u probe/capture_repeat.py 60 > gpurun_out/capture_repeat.log 2>&1
echo "[r03g] capture_repeat rc=$?"; tail -2 gpurun_out/capture_repeat.log
