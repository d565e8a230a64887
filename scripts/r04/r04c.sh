#!/bin/bash
# Round 4: the bench line with the graph-timed roofline (events created before the capture).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --graph-spans gpurun_out/spans_r04c.json > gpurun_out/bench_r04c.json 2> gpurun_out/bench_r04c.err
rc=$?; echo "[r04c] bench rc=$rc"; head -c 2500 gpurun_out/bench_r04c.json; echo; tail -5 gpurun_out/bench_r04c.err
exit $rc
