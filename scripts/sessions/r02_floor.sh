#!/bin/bash
# Per-launch floor inside a hipGraph (tiny kernels back to back) and the config-2 step under HIP runtime
# launch settings (diagnostic, round 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for envs in "" "HIP_FORCE_DEV_KERNARG=1"; do
  echo "== env: ${envs:-default}"
  env $envs timeout -k 10 120 python -u probe/graph_floor.py || exit 1
  env $envs timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/floor_bench.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/floor_bench.json'));print('bench',d['value'],d['ms_per_step'])"
done
