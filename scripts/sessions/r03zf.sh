#!/bin/bash
# Stream priorities for config 4's overlapped chains: depth_net's stream high (TDE_NET_PRIO), the filter-gradient
# stream low (TDE_WGRAD_PRIO), against default priorities.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
    > gpurun_out/ab_r03zf_$tag.json 2> gpurun_out/ab_r03zf_$tag.err
  local rc=$?
  echo "[r03zf] $tag rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03zf_$tag.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
for r in 1 2; do
  run base$r TDE_X=0 || exit 1
  run nethigh$r TDE_NET_PRIO=high || exit 1
  run wglow$r TDE_WGRAD_PRIO=low || exit 1
  run both$r TDE_NET_PRIO=high TDE_WGRAD_PRIO=low || exit 1
done
echo "[r03zf] done"
