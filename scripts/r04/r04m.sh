#!/bin/bash
# Round 4: branch overlap under the segmented (exchange) capture after the fork fix, then the host cost of the step's
# graph replays (probe/launch_cost.py): host-submission-bound or GPU-bound.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py -k "branch" \
  > gpurun_out/tests_r04m.log 2>&1
rc=$?; tail -6 gpurun_out/tests_r04m.log; case $rc in 0|1) ;; *) exit $rc;; esac
for b in off on; do
  BRANCH=$b timeout -k 10 200 python probe/launch_cost.py > gpurun_out/launch_cost_r04m_br$b.txt 2>&1
  r=$?; grep -v amdgpu.ids gpurun_out/launch_cost_r04m_br$b.txt; [ $r -ne 0 ] && exit $r
done
WORKLOAD=config2 timeout -k 10 200 python probe/launch_cost.py > gpurun_out/launch_cost_r04m_c2.txt 2>&1
r=$?; grep -v amdgpu.ids gpurun_out/launch_cost_r04m_c2.txt; [ $r -ne 0 ] && exit $r
exit $rc
