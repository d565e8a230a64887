#!/bin/bash
# Config-4 A/B (filter-gradient stream placement, 64-row WGRAD tiles) on the pieces capture, then the single-graph
# capture bisect ladder (stops at the first failing rung: a segfault ends the call's GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
    > gpurun_out/ab_r03j_$tag.json 2> gpurun_out/ab_r03j_$tag.err
  local rc=$?
  echo "[r03j] $tag rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r03j_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
run base TDE_X=0 || exit 1
run wg_pair TDE_WGRAD_PROGS=pair || exit 1
run wg_single TDE_WGRAD_PROGS=single || exit 1
run wgbm64 TDE_WGRAD_BM64=1 || exit 1
run base2 TDE_X=0 || exit 1
run wg_pair2 TDE_WGRAD_PROGS=pair || exit 1
run wgbm64_2 TDE_WGRAD_BM64=1 || exit 1
for rung in "solo" "twin" "ov" "ov wg" "wg"; do
  for ia in 0 1; do
    TDE_C4_INLINE_ADAM=$ia timeout -k 10 120 python -X faulthandler -u probe/capture_bisect.py $rung \
      > gpurun_out/bisect_r03j.log 2>&1
    rc=$?; echo "[r03j] bisect '$rung' inline=$ia rc=$rc"
    [ $rc -ne 0 ] && { tail -12 gpurun_out/bisect_r03j.log; exit $rc; }
  done
done
echo "[r03j] all rungs passed"
