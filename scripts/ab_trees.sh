#!/bin/bash
# Same-box bench A/B of the current tree against variants/tree_* (Python-side variants; same libtde.so),
# alternating runs.   WL=config2 REPS=2 bash scripts/ab_trees.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export TDE_LIBRARY="$PWD/tf_depth_estimation_amd/libtde.so"
WL=${WL:-config2}
for r in $(seq 1 ${REPS:-2}); do
  for t in . variants/tree_*; do
    timeout -k 10 200 python3 "$t/bench.py" --workload "$WL" --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline ${AB_ARGS:-} \
      > gpurun_out/abt.json 2> gpurun_out/abt.err || { echo "$t rc=$?"; tail -5 gpurun_out/abt.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abt.json')); print('$WL', sys.argv[1], d['ms_per_step'], 'ms/step', d['value'])" "$t"
  done
done
