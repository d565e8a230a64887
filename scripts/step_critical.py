"""Per-queue timeline of one captured step from a rocprofv3 kernel_trace.csv (diagnostic): busy time, span, and
every idle gap longer than GAP us on each queue with the kernel (on any queue) whose end released it -- the
cross-stream waits that make up the step's critical path.
    python scripts/step_critical.py TRACE.csv [GAP_US] [STEP_FROM_END]"""
import collections
import csv
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:56]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gap_us = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["q"] = r.get("Queue_Id") or r.get("Stream_Id")
    rows.sort(key=lambda r: r["s"])
    idx = [i for i, r in enumerate(rows) if "step_begin_kernel" in r["Kernel_Name"]]
    a, b = idx[-back], idx[-back + 1]
    step = rows[a:b]
    t0, t1 = step[0]["s"], rows[b]["s"]
    print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
    byq = collections.defaultdict(list)
    for r in step:
        byq[r["q"]].append(r)
    ends = sorted(step, key=lambda r: r["e"])
    for q, ks in byq.items():
        busy = sum(r["e"] - r["s"] for r in ks) / 1e3
        print(f"\nqueue {q}: {len(ks)} kernels, busy {busy:.1f} us, first {(ks[0]['s'] - t0) / 1e3:.1f} us, "
              f"last end {(ks[-1]['e'] - t0) / 1e3:.1f} us")
        prev = None
        for r in ks:
            if prev is not None and r["s"] - prev["e"] > gap_us * 1e3:
                # the latest kernel end (on another queue) before this start
                rel = None
                for x in ends:
                    if x["e"] > r["s"]:
                        break
                    if x["q"] != q:
                        rel = x
                why = f"after {short(rel['Kernel_Name'])} on q{rel['q']}" if rel else ""
                print(f"   gap {(r['s'] - prev['e']) / 1e3:7.1f} us at {(prev['e'] - t0) / 1e3:8.1f} before "
                      f"{short(r['Kernel_Name'])}  {why}")
            prev = r


if __name__ == "__main__":
    main()
