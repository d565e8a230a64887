"""Summarise rocprofv3 --pmc passes into per-step HBM bytes per kernel family (roofline.traffic).

    python scripts/pmc_traffic.py --fetch DIR_FETCH --write DIR_WRITE --steps S --out profiles/X.json

DIR_* are the -d directories of two separate rocprofv3 runs of the same bench command (FETCH_SIZE and
WRITE_SIZE do not fit one gfx950 pass: 3 + 2 TCC slots of 4).  Per MI355X_MICROARCH.md §HBM:
FETCH_SIZE counts exactly half the bytes of a 16-B-per-lane streaming read on gfx950 (128-B requests
tallied at 64 B), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are in KB.
S = number of training steps the profiled process ran (all dispatches are divided by it)."""
import argparse
import csv
import glob
import json
import os
import re

FAMILIES = [
    ("conv", re.compile(r"igemm\w*_kernel|splitk_reduce\w*_kernel|skinny_kernel|halo_\w*kernel|hwg_\w*kernel")),
    ("bn", re.compile(r"bn_\w+_kernel")),
    ("head", re.compile(r"head_\w+_kernel")),
    ("loss", re.compile(r"smooth2_kernel|l1_kernel|warp_\w+kernel|pose_\w+kernel|cam_loss|resize_area")),
    ("adam", re.compile(r"adam_kernel")),
]


def family(name):
    for fam, rx in FAMILIES:
        if rx.search(name):
            return fam
    return "other"


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "?")
                v = float(row["Counter_Value"])
                t, n = per.get(name, (0.0, 0))
                per[name] = (t + v, n + 1)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    fetch = load(a.fetch, "FETCH_SIZE")
    write = load(a.write, "WRITE_SIZE")
    fams = {}
    for name in set(fetch) | set(write):
        fam = family(name)
        rd = 2.0 * fetch.get(name, (0.0, 0))[0] * 1024 / a.steps
        wr = write.get(name, (0.0, 0))[0] * 1024 / a.steps
        launches = max(fetch.get(name, (0, 0))[1], write.get(name, (0, 0))[1]) / a.steps
        f = fams.setdefault(fam, {"read_bytes_per_step": 0.0, "write_bytes_per_step": 0.0, "launches_per_step": 0.0})
        f["read_bytes_per_step"] += rd
        f["write_bytes_per_step"] += wr
        f["launches_per_step"] += launches
    for f in fams.values():
        f["hbm_bytes_per_step"] = f["read_bytes_per_step"] + f["write_bytes_per_step"]
    out = {"label": a.label, "steps": a.steps,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950 "
                     "16-B/lane read calibration, MI355X_MICROARCH.md §HBM), KB -> bytes, summed per family / steps",
           "families": fams}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
