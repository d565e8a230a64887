"""One captured step's kernel sequence from a rocprofv3 kernel_trace.csv (diagnostic):
duration, gap to the previous kernel's end, grid (workgroups) and name.
    python scripts/step_seq.py TRACE.csv [KERNELS_PER_STEP_MARKER]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "step_begin_kernel"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
prev_end = None
tot = gaps = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    prev_end = e
    wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
    blocks = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(wg, 1)
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0] if not name.startswith("igemm") else name[:60]
    tot += (e - s) / 1e3
    gaps += max(gap, 0)
    print(f"{(e - s) / 1e3:7.1f} {gap:6.1f} {blocks:6d}  {name[:70]}")
print(f"kernels {b - a}  busy {tot:.1f} us  gaps {gaps:.1f} us  span {(prev_end - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us")
