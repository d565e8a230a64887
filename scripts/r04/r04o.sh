#!/bin/bash
# Round 4: config-4 chain launch order and stream roles vs the branch overlap (HW-queue sharing decides which chain
# waits): default order / main chain first (TDE_C4_MAIN_FIRST) / networks swapped (TDE_C4_OV_NET=single), branch on
# and off; then step timelines of the two main-first variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag env... -- branch
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --branch-overlap $BR \
    > gpurun_out/bench_r04o_$tag.json 2> gpurun_out/bench_r04o_$tag.err
  local r=$?; [ $r -ne 0 ] && { tail -3 gpurun_out/bench_r04o_$tag.err; exit $r; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r04o_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  for BR in off on; do
    run base_br${BR}_$rep TDE_X=0
    run mainfirst_br${BR}_$rep TDE_C4_MAIN_FIRST=1
    run ovsingle_br${BR}_$rep TDE_C4_OV_NET=single
  done
done
for b in off on; do
  TDE_C4_MAIN_FIRST=1 BRANCH=$b timeout -k 10 240 python probe/step_timeline.py gpurun_out/timeline_r04o_mf_br$b.txt > gpurun_out/timeline_r04o_mf_br$b.log 2>&1
  r=$?; head -7 gpurun_out/timeline_r04o_mf_br$b.log; [ $r -ne 0 ] && exit $r
done
exit 0
