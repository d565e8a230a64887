#!/bin/bash
# Graph concurrency on this stack (probe/graph_concurrency.py) under the default HIP settings and with graph
# packet capture off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u probe/graph_concurrency.py > gpurun_out/r03s_gc_default.log 2>&1
rc=$?; echo "[r03s] default rc=$rc"; grep "\[graph_conc" gpurun_out/r03s_gc_default.log; [ $rc -ne 0 ] && exit $rc
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u probe/graph_concurrency.py > gpurun_out/r03s_gc_nopkt.log 2>&1
rc=$?; echo "[r03s] nopkt rc=$rc"; grep "\[graph_conc" gpurun_out/r03s_gc_nopkt.log; [ $rc -ne 0 ] && exit $rc
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-secondary \
  > gpurun_out/ab_r03s_nopkt.json 2> gpurun_out/ab_r03s_nopkt.err
echo "[r03s] bench nopkt rc=$? $(python3 -c "import json; d=json.load(open('gpurun_out/ab_r03s_nopkt.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
