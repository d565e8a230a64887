#!/bin/bash
# Round 4: SyncBN bench after the one-launch refactor (error named), then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --sync-bn --no-secondary --no-cpu-baseline > gpurun_out/bench_r04t_syncbn.json 2> gpurun_out/bench_r04t_syncbn.err
rc=$?; [ $rc -ne 0 ] && { grep -v "^frame" gpurun_out/bench_r04t_syncbn.err | grep -i "error\|tde status" | head -8; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04t_syncbn.json'));print('syncbn', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/bench_r04t_default.json 2> gpurun_out/bench_r04t_default.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04t_default.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04t_default.json'));print('default', d['value'], d['ms_per_step'])"
