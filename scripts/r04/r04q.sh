#!/bin/bash
# Round 4: the whole GPU suite on the current tree (grouped BN partials from the producing kernels), then A/B:
# hardware queues per process 2 / 3 / 4 and non-temporal producer stores (variants/libtde_nt.so), alternating x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04q.log 2>&1
rc=$?; tail -4 gpurun_out/tests_r04q.log; echo "[r04q] tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
one() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/bench_r04q_$tag.json 2> gpurun_out/bench_r04q_$tag.err
  local r=$?; [ $r -ne 0 ] && { tail -3 gpurun_out/bench_r04q_$tag.err; exit $r; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r04q_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  one q4_$rep GPU_MAX_HW_QUEUES=4
  one q3_$rep GPU_MAX_HW_QUEUES=3
  one q2_$rep GPU_MAX_HW_QUEUES=2
  one nt_$rep TDE_LIBRARY=$PWD/variants/libtde_nt.so
done
exit $rc
