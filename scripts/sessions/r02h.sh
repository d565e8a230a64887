#!/bin/bash
# Filter-gradient side-stream overlap: A/B on configs 2/3/4, then the trainer/DDP GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in config2 config4 config3; do
for ov in off on; do
  timeout -k 10 200 python -u bench.py --workload $wl --steps 30 --warmup 10 --no-cpu-baseline --wgrad-overlap $ov > gpurun_out/r02h_bench.json 2>gpurun_out/r02h_bench.err || { tail -20 gpurun_out/r02h_bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02h_bench.json'));print('$wl $ov',d['value'],d['ms_per_step'],d['final_loss'])"
done; done
