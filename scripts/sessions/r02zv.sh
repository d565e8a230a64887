#!/bin/bash
# Round-2 final measurements (session 6 tree): conv-family HBM traffic (two PMC passes, config 2), full GPU
# suite + smoke, bench.py (with its CPU baseline) on all four workloads, kernel traces of configs 2 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r02zv
bash scripts/pmc.sh $TAG config2 fp16x3 8 || exit $?
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
for WL in config2 config3 config4 config5; do
  timeout -k 10 300 python -u bench.py --workload $WL > gpurun_out/bench_${TAG}_$WL.json 2> gpurun_out/bench_${TAG}_$WL.err || { tail -5 gpurun_out/bench_${TAG}_$WL.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$WL.json'));print('$WL',d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'],d.get('depth_l1_vs_ref',{}).get('worst_max_rel'))"
done
for WL in config2 config4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_$WL" -o run --output-format csv \
    -- python3 bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}_$WL.log 2>&1 || exit $?
  echo "prof $WL ok"
done
