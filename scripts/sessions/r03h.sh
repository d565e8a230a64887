#!/bin/bash
# A/B: HW queue count (2 / 3 / 4), inline Adam; then the single-graph capture crash under faulthandler + HIP log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
    > gpurun_out/ab_r03h_$tag.json 2> gpurun_out/ab_r03h_$tag.err
  local rc=$?
  echo "[r03h] $tag rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r03h_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
run base TDE_X=0 || exit 1
run q3 GPU_MAX_HW_QUEUES=3 || exit 1
run q2 GPU_MAX_HW_QUEUES=2 || exit 1
run noinline TDE_C4_INLINE_ADAM=0 || exit 1
run bm128 TDE_BM64_MAXM=0 || exit 1
run bm64le1536 TDE_BM64_MAXM=1536 || exit 1
run base2 TDE_X=0 || exit 1
# the single-graph capture: Python stack at the fault + the last HIP API calls
AMD_LOG_LEVEL=3 timeout -k 10 120 python -X faulthandler -u probe/capture_repeat.py 2 > gpurun_out/capture_single.log 2> gpurun_out/capture_single.err
echo "[r03h] capture probe rc=$?"
tail -c 20000 gpurun_out/capture_single.err > gpurun_out/capture_single_tail.err
rm -f gpurun_out/capture_single.err
tail -3 gpurun_out/capture_single.log
exit 0
