#!/bin/bash
# Is config 4's two-stream piece replay concurrent?  The same piece graphs replayed on two streams (default) vs one
# after another on one stream (TDE_C4_OV_SERIAL=1), without the profiler.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    TDE_C4_OV_SERIAL=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r03zd_ser$v$r.json 2> gpurun_out/ab_r03zd_ser$v$r.err
    rc=$?; echo "[r03zd] serial=$v/$r rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03zd_ser$v$r.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo "[r03zd] done"
