"""One training step from a rocprofv3 kernel trace: dispatch order, grid, duration and the idle gap
before each kernel (diagnostic).   python scripts/trace_step.py run_kernel_trace.csv [--top N]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
a, b = adam[-2], adam[-1]
step = rows[a + 1:b + 1]
t0 = int(step[0]["Start_Timestamp"])
t1 = int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"step: {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
      f"gaps {(t1 - t0 - busy) / 1e3:.1f} us")


def short(n):
    m = re.search(r"::(\w+)(<[^>(]*>)?\(", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


out = []
prev_end = None
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) if prev_end is not None else 0
    prev_end = e
    grid = f"{int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    out.append(((e - s) / 1e3, gap / 1e3, short(r["Kernel_Name"]), grid))
for d, g, n, grid in sorted(out, reverse=True)[:top]:
    print(f"{d:8.1f} us  gap {g:6.1f}  {n:50s} grid {grid}")
