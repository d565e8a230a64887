#!/bin/bash
# A/B of planner environment knobs on config 4 (and config 2), alternating on one box.  Arguments: variants as
# NAME=VALUE[,NAME=VALUE] strings; "base" = no variable.  TAG names the output files.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04f}
for rep in 1 2; do
  for v in "$@"; do
    for w in config4 config2; do
      envs=""; [ "$v" != "base" ] && envs=$(echo "$v" | tr ',' ' ')
      f=gpurun_out/ab_${TAG}_${w}_$(echo "$v" | tr '=,' '__')_$rep.json
      env $envs timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-secondary > $f 2>/dev/null
      rc=$?; [ $rc -ne 0 ] && { echo "$v $w rc=$rc"; exit $rc; }
      python -c "import json;d=json.load(open('$f'));print('$w $v rep $rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
    done
  done
done
