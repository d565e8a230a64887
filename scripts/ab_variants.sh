#!/bin/bash
# conv_micro under each variants/libtde_*.so (diagnostic A/B; one process per variant).
#   bash scripts/ab_variants.sh "shape1,shape2" [modes] [math]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SH=${1:-}; MODES=${2:-fwd,dgrad,wgrad}; MATH=${3:-fp32}
for so in variants/libtde_*.so; do
  v=$(basename "$so" .so)
  TDE_LIBRARY="$PWD/$so" timeout -k 10 120 python3 scripts/conv_micro.py --math "$MATH" --shapes "$SH" --modes "$MODES" \
    --reps 30 > "gpurun_out/ab_$v.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 "gpurun_out/ab_$v.log"; exit $rc; }
  echo "== $v"; grep -v "^==\|amdgpu.ids" "gpurun_out/ab_$v.log"
done
if [ "${AB_BENCH:-0}" = "1" ]; then
  for so in variants/libtde_*.so; do
    v=$(basename "$so" .so)
    TDE_LIBRARY="$PWD/$so" timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline \
      ${AB_BENCH_ARGS:-} > "gpurun_out/abb_$v.json" 2> "gpurun_out/abb_$v.err"
    rc=$?; [ $rc -ne 0 ] && { echo "$v bench rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], 'ms/step', d['value'], d['roofline']['achieved'], 'TF conv')" "gpurun_out/abb_$v.json" "$v"
  done
fi
