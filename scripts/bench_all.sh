#!/bin/bash
# Bench every BASELINE workload on one GPU (each step under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-30}
for w in config2 config4 config3 config5; do
  timeout -k 10 400 python bench.py --workload $w --steps "$STEPS" --warmup 5 ${BENCH_ARGS:-} \
    > gpurun_out/bench_${TAG}_$w.json 2> gpurun_out/bench_${TAG}_$w.err
  rc=$?
  echo "[bench_all] $w rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_${TAG}_$w.err; exit $rc; fi
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms/step', 'conv', d['roofline']['achieved'], 'TF/s', 'cpu', d.get('cpu_baseline',{}).get('value'))" gpurun_out/bench_${TAG}_$w.json $w
done
