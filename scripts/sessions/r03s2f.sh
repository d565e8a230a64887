#!/bin/bash
# Two-chain config-4 schedule: knob re-check (which network on the second stream, filter-gradient stream count,
# which programs' filter gradients go to a side stream), alternating x2, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {   # tag, env..., -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary "$@" > gpurun_out/ab_r03s2f_$tag.json 2>/dev/null
  local rc=$?; [ $rc -ne 0 ] && { echo "$tag rc=$rc"; exit $rc; }
  echo "$tag: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03s2f_$tag.json')); print(d['value'], d['ms_per_step'])")"
}
for i in 1 2; do
  run base_$i X=1 --
  run ovsingle_$i TDE_C4_OV_NET=single --
  run wgs2_$i TDE_WGRAD_STREAMS=2 --
  run wgall_$i X=1 -- --wgrad-progs all
done
