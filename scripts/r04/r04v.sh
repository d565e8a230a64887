#!/bin/bash
# Round 4: same-box A/B of build variants (variants/libtde_*.so: BN apply grid: rows per lane 8 / 4 / 16),
# alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in cur rpl4 rpl16; do
    TDE_LIBRARY="$PWD/variants/libtde_$v.so" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary \
      > gpurun_out/ab_r04v_${v}_$rep.json 2> gpurun_out/ab_r04v_${v}_$rep.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/ab_r04v_${v}_$rep.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_r04v_${v}_$rep.json $v
  done
done
