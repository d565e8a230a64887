#!/bin/bash
# Config 4: the filter-gradient placement default (depth_net's only) vs the other net on the second stream; then
# the single-graph capture rungs that test the nested-fork hypothesis (expected-to-pass first; the nested fork
# -- capture stream -> depth_net's stream -> its filter-gradient stream -- last, as it may segfault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
    > gpurun_out/ab_r03k_$tag.json 2> gpurun_out/ab_r03k_$tag.err
  local rc=$?
  echo "[r03k] $tag rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r03k_$tag.json')); print(d['value'], d['ms_per_step'], d['config'].get('wgrad_progs'))" 2>/dev/null)"
  return $rc
}
run base TDE_X=0 || exit 1
run ovs_wgp TDE_C4_OV_NET=single TDE_WGRAD_PROGS=pair || exit 1
run ovs_wgs TDE_C4_OV_NET=single TDE_WGRAD_PROGS=single || exit 1
run base2 TDE_X=0 || exit 1
run wg_all TDE_WGRAD_PROGS=single,pair || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/r03k_tests.log 2>&1
rc=$?; echo "[r03k] tests rc=$rc"; tail -3 gpurun_out/r03k_tests.log; [ $rc -ne 0 ] && exit $rc
for rung in "ov wgs" "ovs wgp"; do
  timeout -k 10 120 python -X faulthandler -u probe/capture_bisect.py $rung > gpurun_out/bisect_r03k.log 2>&1
  rc=$?; echo "[r03k] bisect '$rung' rc=$rc"; [ $rc -ne 0 ] && { tail -8 gpurun_out/bisect_r03k.log; exit $rc; }
done
run single_ovs_wgp TDE_C4_OV_NET=single TDE_WGRAD_PROGS=pair TDE_C4_SINGLE_GRAPH=1 || exit 1
timeout -k 10 120 python -X faulthandler -u probe/capture_bisect.py ov wgp > gpurun_out/bisect_r03k.log 2>&1
rc=$?; echo "[r03k] bisect 'ov wgp' rc=$rc"; tail -3 gpurun_out/bisect_r03k.log
