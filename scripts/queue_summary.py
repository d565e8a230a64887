"""Per-queue kernel time by kernel name for one captured step of a rocprofv3 kernel_trace.csv (diagnostic).
    python scripts/queue_summary.py TRACE.csv [TOP]"""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "step_begin_kernel" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
step = rows[a:b]
qs = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
for r in step:
    q = r.get("Queue_Id") or r.get("Stream_Id")
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0][:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    qs[q][n][0] += 1; qs[q][n][1] += d
for q, m in qs.items():
    tot = sum(v[1] for v in m.values())
    print(f"queue {q}: {tot:.1f} us")
    for n, (c, d) in sorted(m.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
        print(f"   {d:8.1f} us  {c:3d}x  {n}")
