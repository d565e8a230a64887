#!/bin/bash
# Round 4: one-launch SyncBN phases -- the kernel / grouped-BN tests, the DDP suites, then the SyncBN bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "syncbn or grouped or fused_bn or bn_train" --timeout 300 --timeout-method thread > gpurun_out/tests_r04s_k.log 2>&1
rc=$?; tail -4 gpurun_out/tests_r04s_k.log; echo "[r04s] kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_ddp_world2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04s_ddp.log 2>&1
rc=$?; tail -4 gpurun_out/tests_r04s_ddp.log; echo "[r04s] ddp tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --sync-bn --no-secondary --no-cpu-baseline > gpurun_out/bench_r04s_syncbn.json 2> gpurun_out/bench_r04s_syncbn.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04s_syncbn.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04s_syncbn.json'));print('syncbn', d['value'], d['ms_per_step'], d['config'])"
