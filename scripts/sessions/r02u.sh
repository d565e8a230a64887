#!/bin/bash
# Single-launch ticketed BN (bn_fused_kernel): GPU tests, then a TDE_BN_FUSED on/off bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02u}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${TESTS:-} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for WL in ${WLS:-config2}; do
for r in 1 2; do
for f in 0 1; do
  TDE_BN_FUSED=$f timeout -k 10 200 python -u bench.py --workload $WL --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_b.json'));print('$WL fused $f',d['value'],d['ms_per_step'], d['depth_l1_vs_ref']['worst_max_rel'] if 'depth_l1_vs_ref' in d else '')"
done
done
done
