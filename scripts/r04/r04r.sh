#!/bin/bash
# Round 4: the rest of the GPU suite after the grouped-BN test fix, then HW queues 5 / 6 vs 4 (alternating x2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04r.log 2>&1
rc=$?; tail -4 gpurun_out/tests_r04r.log; echo "[r04r] tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
one() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/bench_r04r_$tag.json 2> gpurun_out/bench_r04r_$tag.err
  local r=$?; [ $r -ne 0 ] && { tail -3 gpurun_out/bench_r04r_$tag.err; exit $r; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r04r_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  one q4_$rep GPU_MAX_HW_QUEUES=4
  one q5_$rep GPU_MAX_HW_QUEUES=5
  one q6_$rep GPU_MAX_HW_QUEUES=6
done
exit $rc
