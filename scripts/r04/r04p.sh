#!/bin/bash
# Round 4: kernel statistics of the default bench (config 4) on the current tree (rocprofv3 --kernel-trace --stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r04p" -o run --output-format csv \
  -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/prof_r04p.log 2>&1
rc=$?; echo "[r04p] rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_r04p.log; exit $rc; }
f=$(find gpurun_out/prof_r04p -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r04p_config4_kernel_stats.csv
# steps in the trace: 2 eager (plain + instrumented) + 7 graph-timed replays + 2 capture warm-ups + 5 warm-up + 30 timed
python3 scripts/kstats.py gpurun_out/r04p_config4_kernel_stats.csv 46 60
