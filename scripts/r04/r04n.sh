#!/bin/bash
# Round 4: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) vs the config-4 step's concurrent streams:
# the bench and the step timeline at 4 / 8 / 16 queues, branch overlap on and off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for q in 4 8 16; do
  for b in on off; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --branch-overlap $b --no-secondary --no-cpu-baseline \
      > gpurun_out/bench_r04n_q${q}_br$b.json 2> gpurun_out/bench_r04n_q${q}_br$b.err
    r=$?; [ $r -ne 0 ] && { tail -3 gpurun_out/bench_r04n_q${q}_br$b.err; exit $r; }
    python -c "import json;d=json.load(open('gpurun_out/bench_r04n_q${q}_br$b.json'));print('queues $q branch $b', d['value'], d['ms_per_step'])"
  done
done
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q BRANCH=on timeout -k 10 240 python probe/step_timeline.py gpurun_out/timeline_r04n_q$q.txt > gpurun_out/timeline_r04n_q$q.log 2>&1
  r=$?; head -8 gpurun_out/timeline_r04n_q$q.log; [ $r -ne 0 ] && exit $r
done
exit 0
