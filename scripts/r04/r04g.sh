#!/bin/bash
# Round 4: capturable, row-grouped SyncBN (world-1 RCCL capture test, world-2 gloo config-4 SyncBN), the bench with
# --sync-bn (graph) against the default, then planner-knob A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py \
  tests/test_gpu_ddp_world2.py > gpurun_out/tests_r04g.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/tests_r04g.log | tail -20; echo "[r04g] tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for sb in "" "--sync-bn"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary $sb > gpurun_out/bench_r04g$sb.json 2> gpurun_out/bench_r04g$sb.err
  rc2=$?; echo "[r04g] bench $sb rc=$rc2"; [ $rc2 -ne 0 ] && { tail -4 gpurun_out/bench_r04g$sb.err; exit $rc2; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r04g$sb.json'));print('$sb', d['value'], d['ms_per_step'], d['config']['hip_graph'], d['config']['batch_norm'])"
done
[ $rc -ne 0 ] && exit $rc
TAG=r04f bash scripts/r04/ab_env.sh base TDE_DECONV_PS_MINBLOCKS=192 TDE_BM64_MAXM=16384 TDE_SPLIT_MINKT=6
