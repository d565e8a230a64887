#!/bin/bash
# bench.py under several environment settings (diagnostic A/B of host-side tuning knobs).
#   bash scripts/ab_env.sh "NAME1:VAR=V VAR2=V" "NAME2:..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline ${AB_BENCH_ARGS:-} \
    > "gpurun_out/abe_$name.json" 2> "gpurun_out/abe_$name.err"
  rc=$?; [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -3 "gpurun_out/abe_$name.err"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_breakdown_ms']; print(sys.argv[2], d['ms_per_step'], 'ms/step conv', d['roofline']['conv_ms_per_step'], 'fwd', k.get('conv_fwd'), 'bwd', k.get('conv_bwd'), 'wgrad', k.get('conv_wgrad'))" "gpurun_out/abe_$name.json" "$name"
done
