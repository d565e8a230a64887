"""Per-queue busy time and gaps of one captured step from a rocprofv3 kernel_trace.csv (diagnostic): shows which
HW queue (graph branch) carries the critical path and how much of it is idle between its own kernels.
    python scripts/stream_gaps.py TRACE.csv [MARKER] [TOPN]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "step_begin_kernel"
topn = int(sys.argv[3]) if len(sys.argv) > 3 else 15
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
byq = collections.defaultdict(list)
for r in step:
    byq[r["Queue_Id"]].append(r)
print(f"span {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
for q, rs in byq.items():
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
    gaps = []
    for p, r in zip(rs, rs[1:]):
        g = (int(r["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3
        gaps.append((g, p["Kernel_Name"][:50], r["Kernel_Name"][:50]))
    tot = sum(g for g, _, _ in gaps if g > 0)
    big = sum(g for g, _, _ in gaps if g > 2.5)
    print(f"queue {q}: {len(rs)} kernels, busy {busy:.1f} us, gaps {tot:.1f} us (>2.5us: {big:.1f} us in "
          f"{sum(1 for g, _, _ in gaps if g > 2.5)})")
    for g, p, n in sorted(gaps, reverse=True)[:topn]:
        print(f"    {g:7.1f}  {p.replace('(anonymous namespace)::', '')[:40]:40s} -> {n.replace('(anonymous namespace)::', '')[:40]}")
