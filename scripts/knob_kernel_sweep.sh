#!/bin/bash
# One tuning knob swept under rocprofv3: average duration of the kernels whose name contains PATTERN.
#   bash scripts/knob_kernel_sweep.sh KNOB PATTERN "workload ..." "value ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KNOB=$1; PAT=$2; WLS=$3; VALS=$4
for w in $WLS; do for b in $VALS; do
  d="$PWD/gpurun_out/prof_knob_${w}_$(basename "$b")"
  env "$KNOB=$b" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
    -- python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > "$d.log" 2>&1 || exit 1
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r['Name']: print(sys.argv[3], sys.argv[4], '%8.2f us avg %5s calls' % (float(r['AverageNs'])/1e3, r['Calls']), r['Name'][:40])
" "$f" "$PAT" "$w" "$KNOB=$b"
  rm -rf "$d"
done; done
