#!/bin/bash
# A/B on one box: HEAD-of-round tree (variants/tree_base) vs the current tree at TDE_WGRAD_TAIL 0/1/2/4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export TDE_LIBRARY="$PWD/tf_depth_estimation_amd/libtde.so"
for WL in ${WLS:-config2}; do
for r in 1 2; do
  for v in base t0 t1 t2 t4; do
    if [ $v = base ]; then b=variants/tree_base/bench.py; e=""; else b=bench.py; e="TDE_WGRAD_TAIL=${v#t}"; fi
    env $e timeout -k 10 200 python3 $b --workload $WL --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/abt.json 2> gpurun_out/abt.err || { echo "$v rc=$?"; tail -5 gpurun_out/abt.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abt.json')); print('$WL $v', d['ms_per_step'], 'ms/step', d['value'])"
  done
done
done
