#!/bin/bash
# Stream-priority A/B (experiment knobs TDE_REPLAY_PRIO / TDE_WGRAD_PRIO) on the config-2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python - <<'PY' || exit 1
import torch
print("priority range", torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else None)
PY
for r in 1 2; do
for e in "X=0" "TDE_REPLAY_PRIO=-1" "TDE_WGRAD_PRIO=1" "TDE_REPLAY_PRIO=-1 TDE_WGRAD_PRIO=1"; do
  env $e timeout -k 10 200 python -u bench.py --workload ${WL:-config2} --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r02w_b.json 2>gpurun_out/r02w_b.err || { tail -5 gpurun_out/r02w_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02w_b.json'));print('$e',d['value'],d['ms_per_step'])"
done
done
for r in 1 2; do
for e in "X=0" "TDE_WARP_MAXB=100000"; do
  env $e timeout -k 10 200 python -u bench.py --workload config4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02w_b.json 2>gpurun_out/r02w_b.err || { tail -5 gpurun_out/r02w_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02w_b.json'));print('config4 $e',d['value'],d['ms_per_step'])"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r02w_config2" -o run --output-format csv \
  -- python3 bench.py --workload config2 --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/prof_r02w_config2.log 2>&1 || { echo "rocprofv3 failed"; exit 1; }
