#!/bin/bash
# BN backward partial-row count A/B (TDE_BN_MAXCH: row chunks of bn_part_kernel<1>) on config 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for m in 1024 256 64 32; do
  TDE_BN_MAXCH=$m timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r02zd_b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02zd_b.json'));print('maxch $m',d['value'],d['ms_per_step'],d['kernel_breakdown_ms']['bn_bwd'])"
done
done
