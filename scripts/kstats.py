"""Per-step kernel time table from a rocprofv3 --stats kernel_stats.csv (diagnostic).
    python scripts/kstats.py CSV STEPS [TOP]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e3 / steps:8.1f} us/step {int(r['Calls']) / steps:5.1f}/step "
          f"{float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:80]}")
print("total ms/step", sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / steps)
