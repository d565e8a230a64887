#!/bin/bash
# Fused pose gradient: trainer/DDP/full-size GPU tests; then filter-gradient placement knobs (group, tail, inline rows), alternating x2, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainers.py tests/test_gpu_ddp.py tests/test_gpu_fullsize.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/tests_r03s2g.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r03s2g.log; [ $rc -ne 0 ] && exit $rc
run() {   # tag, env..., -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary "$@" > gpurun_out/ab_r03s2g_$tag.json 2>/dev/null
  local rc=$?; [ $rc -ne 0 ] && { echo "$tag rc=$rc"; exit $rc; }
  echo "$tag: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03s2g_$tag.json')); print(d['value'], d['ms_per_step'])")"
}
for i in 1 2; do
  run base_$i X=1 --
  run group2_$i TDE_WGRAD_GROUP=2 --
  run tail2_$i TDE_WGRAD_TAIL=2 --
  run tail3_$i TDE_WGRAD_TAIL=3 --
  run inl6k_$i TDE_WGRAD_INLINE_M=6144 --
done
