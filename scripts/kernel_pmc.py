"""Per-kernel means of rocprofv3 --pmc counters (diagnostic): every *counter_collection.csv under the given dirs,
grouped by kernel name (substring filter) and counter, averaged per dispatch.

    python scripts/kernel_pmc.py DIR [DIR ...] [--filter hwh_kernel]"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    per = {}
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "?")
                    if a.filter not in name:
                        continue
                    key = (name[:90], row["Counter_Name"])
                    t, n = per.get(key, (0.0, 0))
                    per[key] = (t + float(row["Counter_Value"]), n + 1)
    last = None
    for (name, ctr), (t, n) in sorted(per.items()):
        if name != last:
            print(name)
            last = name
        print(f"    {ctr:28s} {t / n:16.1f}   (n={n})")


if __name__ == "__main__":
    main()
