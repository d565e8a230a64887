#!/bin/bash
# Round 4: capture-crash reproducer (plain HIP), the new GPU tests (world-2 on one GPU, B=8 config-4 parity,
# deferred-Adam mid-run flush, conv bwd-data pixel shuffle), then the bench line with the graph-timed roofline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/capture_fork2_r04b.txt
for v in 1 2 3 4 5 6; do
  timeout -k 5 60 ./probe/capture_fork2 $v >> gpurun_out/capture_fork2_r04b.txt 2>&1
  rc=$?; echo "variant $v exit $rc" >> gpurun_out/capture_fork2_r04b.txt
  case $rc in 0|1|2) ;; *) echo "[r04b] probe variant $v rc=$rc: stopping GPU work"; cat gpurun_out/capture_fork2_r04b.txt; exit $rc;; esac
done
cat gpurun_out/capture_fork2_r04b.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ddp_world2.py tests/test_gpu_fullsize.py::test_config4_forward_benched_batch \
  "tests/test_gpu_trainers.py::test_deferred_adam_matches_plain" tests/test_gpu_kernels.py -k "pixel_shuffle or deferred or world or benched" \
  > gpurun_out/tests_r04b.log 2>&1
rc=$?; tail -25 gpurun_out/tests_r04b.log; echo "[r04b] tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench_r04b.json 2> gpurun_out/bench_r04b.err
rc2=$?; echo "[r04b] bench rc=$rc2"; head -c 1500 gpurun_out/bench_r04b.json; echo
exit $((rc2 != 0 ? rc2 : rc))
