#!/bin/bash
# Round 4 closing evidence of the final tree: the whole GPU suite, smoke(), the default bench line, its kernel
# statistics (rocprofv3 --kernel-trace --stats) and the conv family's PMC traffic (three separate counter passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04w.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r04w.log; echo "[r04w] tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04w.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_r04w.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r04w.json 2> gpurun_out/bench_r04w.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04w.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04w.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r04w" -o run --output-format csv \
  -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/prof_r04w.log 2>&1
rc=$?; echo "[r04w] rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_r04w.log; exit $rc; }
f=$(find gpurun_out/prof_r04w -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r04w_config4_kernel_stats.csv
rm -rf gpurun_out/prof_r04w
python3 scripts/kstats.py gpurun_out/r04w_config4_kernel_stats.csv 46 40 > gpurun_out/r04w_kstats.txt
tail -1 gpurun_out/r04w_kstats.txt
bash scripts/pmc_step.sh r04w config4
rc=$?; echo "[r04w] pmc rc=$rc"
exit $rc
