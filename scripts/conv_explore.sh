#!/bin/bash
# Kernel-only times (rocprofv3 kernel trace) of one conv shape/mode over tile, split and prefetch
# overrides (diagnostic).   bash scripts/conv_explore.sh SHAPE MODE "BN:SPLITS:PF:BM ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SH=$1; MODE=$2; CFGS=$3
for c in $CFGS; do
  IFS=: read bn sp pf bm <<< "$c"
  d="$PWD/gpurun_out/cx_${SH}_${MODE}_$c"
  TDE_FORCE_BN=$bn TDE_FORCE_SPLITS=$sp TDE_CONV_PF=$pf TDE_FORCE_BM=$bm timeout -k 10 120 rocprofv3 --kernel-trace -d "$d" -o run \
    --output-format csv -- python3 scripts/conv_micro.py --math fp32 --shapes "$SH" --modes "$MODE" --reps 20 > "$d.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$c rc=$rc"; tail -3 "$d.log"; exit $rc; }
  python3 - "$d" "$c" <<'PY'
import csv, glob, sys, collections
d, c = sys.argv[1], sys.argv[2]
t = collections.defaultdict(list)
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]; k = "igemm" if "igemmx" in n else ("reduce" if "reduce" in n else n[:20])
        t[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(c, "  ".join(f"{k} {sorted(v)[len(v) // 2]:.1f}us x{len(v)}" for k, v in t.items()))
PY
done
