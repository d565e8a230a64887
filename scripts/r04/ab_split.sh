#!/bin/bash
# A/B of the split-K block target on config 4 (and config 2), alternating on one box: TDE_SPLIT_TARGET values given
# as arguments (default 512 384).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04e}
VALS=${*:-512 384}
for rep in 1 2; do
  for t in $VALS; do
    for w in config4 config2; do
      TDE_SPLIT_TARGET=$t timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-secondary \
        > gpurun_out/ab_${TAG}_${w}_split${t}_$rep.json 2>/dev/null
      rc=$?; [ $rc -ne 0 ] && { echo "split $t $w rc=$rc"; exit $rc; }
      python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_${w}_split${t}_$rep.json'));print('$w split $t rep $rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
    done
  done
done
