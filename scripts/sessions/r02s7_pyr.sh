#!/bin/bash
# Depth-pyramid loss head: full-resolution scale with four pixels per round (loss.hip) vs the one-pixel loop
# (variants/libtde_pyr0.so): loss-kernel GPU tests, rocprofv3 kernel time of each build, alternating benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
X0="TDE_LIBRARY=$PWD/variants/libtde_pyr0.so"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainers.py -q -m gpu -k "pyramid or loss or config" \
  --timeout 120 --timeout-method thread > gpurun_out/pyr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pyr_tests.log; [ $rc -ne 0 ] && exit $rc
for v in p1 p0; do
  if [ $v = p0 ]; then export TDE_LIBRARY=$PWD/variants/libtde_pyr0.so; else unset TDE_LIBRARY; fi
  for w in config2 config4; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_pyr${v}_$w" -o run --output-format csv \
      -- python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_pyr${v}_$w.log 2>&1 || exit 1
    f=$(find gpurun_out/prof_pyr${v}_$w -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pyramid' in r['Name']: print(sys.argv[2], '%8.2f us avg %5s calls' % (float(r['AverageNs'])/1e3, r['Calls']), r['Name'][:50])
" "$f" "$v $w"
  done
done
unset TDE_LIBRARY
bash scripts/ab_env.sh "p1:TDE_X=0" "p0:$X0" "p1b:TDE_X=0" "p0b:$X0" || exit 1
