#!/bin/bash
# Round 4, re-entry session: the branch-overlap tests (depth_net's pose / mask branches on their own stream), the
# whole GPU suite + smoke, the bench line with and without the branch overlap, then the family-skip upper bounds of
# the config-4 step (probe/skip_family.py: what each kernel family costs the critical path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { case $1 in 0|1) return 0;; *) echo "[r04l] $2 rc=$1: stopping GPU work"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trainers.py tests/test_gpu_ddp.py \
  -k "branch or sync_bn_captured" > gpurun_out/tests_r04l_branch.log 2>&1
rcb=$?; tail -8 gpurun_out/tests_r04l_branch.log; ok $rcb "branch tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04l.log 2>&1
rc=$?; tail -4 gpurun_out/tests_r04l.log; echo "[r04l] tests rc=$rc"; ok $rc "gpu suite"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04l.txt 2>&1
rc1=$?; tail -1 gpurun_out/smoke_r04l.txt; [ $rc1 -ne 0 ] && exit $rc1
for b in on off; do
  timeout -k 10 600 python bench.py --branch-overlap $b $([ $b = off ] && echo --no-secondary --no-cpu-baseline) \
    > gpurun_out/bench_r04l_br$b.json 2> gpurun_out/bench_r04l_br$b.err
  rc2=$?; echo "[r04l] bench branch=$b rc=$rc2"; [ $rc2 -ne 0 ] && { tail -5 gpurun_out/bench_r04l_br$b.err; ok $rc2 bench; continue; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r04l_br$b.json'));print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac']);print(d.get('secondary'))"
done
timeout -k 10 600 python bench.py --sync-bn --no-secondary --no-cpu-baseline > gpurun_out/bench_r04l_syncbn.json 2> gpurun_out/bench_r04l_syncbn.err
rc5=$?; echo "[r04l] bench syncbn rc=$rc5"; ok $rc5 "syncbn bench"
[ $rc5 -eq 0 ] && python -c "import json;d=json.load(open('gpurun_out/bench_r04l_syncbn.json'));print('syncbn value',d['value'],'ms',d['ms_per_step'],d['config'])"
: > gpurun_out/skip_r04l.txt
for s in "" bnf bnb bnf,bnb head warp,pyr adam resize,copy; do
  SKIP=$s timeout -k 10 180 python probe/skip_family.py 100 >> gpurun_out/skip_r04l.txt 2>/dev/null
  rc3=$?; [ $rc3 -ne 0 ] && { echo "[r04l] skip '$s' rc=$rc3"; cat gpurun_out/skip_r04l.txt; exit $rc3; }
done
cat gpurun_out/skip_r04l.txt
for b in on off; do
  BRANCH=$b timeout -k 10 240 python probe/step_timeline.py gpurun_out/timeline_r04l_br$b.txt > gpurun_out/timeline_r04l_br$b.log 2>&1
  rc4=$?; head -60 gpurun_out/timeline_r04l_br$b.log; [ $rc4 -ne 0 ] && exit $rc4
done
exit $((rcb != 0 ? rcb : rc))
