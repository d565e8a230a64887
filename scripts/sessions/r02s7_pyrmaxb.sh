#!/bin/bash
# depth_pyramid_kernel block cap per scale (TDE_PYR_MAXB) re-swept on the current tree: rocprofv3 kernel time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in config2 config4; do for b in 128 160 192 224 192 128; do
  export TDE_PYR_MAXB=$b
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_pmb${w}_$b" -o run --output-format csv \
    -- python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_pmb${w}_$b.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_pmb${w}_$b -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pyramid' in r['Name']: print(sys.argv[3], 'maxb', sys.argv[2], '%8.2f us avg %5s calls' % (float(r['AverageNs'])/1e3, r['Calls']))
" "$f" "$b" "$w"
  rm -rf gpurun_out/prof_pmb${w}_$b
done; done
