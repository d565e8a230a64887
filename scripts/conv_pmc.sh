#!/bin/bash
# SQ/MFMA counters of one conv micro shape (diagnostic).  bash scripts/conv_pmc.sh SHAPE MODE [TAG]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SH=$1; MODE=$2; TAG=${3:-x}; MATH=${MATH:-fp32}; KPAT=${KPAT:-igemmx}
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_SALU"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace -d "$PWD/gpurun_out/cpmc_${TAG}_$i" -o run --output-format csv \
    -- python3 scripts/conv_micro.py --math $MATH --shapes "$SH" --modes "$MODE" --reps 5 > "gpurun_out/cpmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "[conv_pmc] set $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - "$TAG" "$KPAT" <<'PY'
import csv, glob, sys, collections
tag, kpat = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: [0.0, 0])
for f in glob.glob(f"gpurun_out/cpmc_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kpat not in r["Kernel_Name"]:
            continue
        a = agg[r["Counter_Name"]]
        a[0] += float(r["Counter_Value"]); a[1] += 1
for k, (v, n) in sorted(agg.items()):
    print(f"{k:28s} {v / max(n, 1):16.1f}  (avg over {n} dispatches)")
PY
