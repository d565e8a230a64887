#!/bin/bash
# New-feature GPU tests (nets.disp_net, BN-free pairtest disp_net, K=3 heads, bias+ReLU backward), then the
# round-3 profiling session (scripts/sessions/r03a.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nets.py tests/test_gpu_kernels.py -x -q --timeout 120 \
  --timeout-method thread -k "sfm or bn_free or bias_relu or head_fwd_bwd or resize_fwd_bwd" > gpurun_out/r03b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03b_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/sessions/r03a.sh
