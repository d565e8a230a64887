#!/bin/bash
# Capture-safe events: the single-graph capture probe (60 captures in one process), the config-4 bench with
# the single graph vs the pieces, and the GPU tests touched by the change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -X faulthandler -u probe/capture_repeat.py 60 > gpurun_out/capture_repeat.log 2>&1
rc=$?; echo "[r03i] capture_repeat rc=$rc"; tail -2 gpurun_out/capture_repeat.log
[ $rc -ne 0 ] && exit $rc
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
    > gpurun_out/ab_r03i_$tag.json 2> gpurun_out/ab_r03i_$tag.err
  local rc=$?
  echo "[r03i] $tag rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r03i_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
run pieces TDE_X=0 || exit 1
run single TDE_C4_SINGLE_GRAPH=1 || exit 1
run wg_pair TDE_WGRAD_PROGS=pair || exit 1
run wg_single TDE_WGRAD_PROGS=single || exit 1
run single_wg_pair TDE_C4_SINGLE_GRAPH=1 TDE_WGRAD_PROGS=pair || exit 1
run pieces2 TDE_X=0 || exit 1
run single2 TDE_C4_SINGLE_GRAPH=1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_inference.py -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1
echo "[r03i] tests rc=$?"; tail -3 gpurun_out/r03i_tests.log
