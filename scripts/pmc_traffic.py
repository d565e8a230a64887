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
    ("conv", re.compile(r"igemm\w*_kernel|ring_\w*kernel|splitk_reduce\w*_kernel|skinny_kernel|halo_\w*kernel|hwg_\w*kernel|hwh_\w*kernel")),
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
    ap.add_argument("--sq", default=None, help="dir of a third pass with SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE")
    a = ap.parse_args()
    fetch = load(a.fetch, "FETCH_SIZE")
    write = load(a.write, "WRITE_SIZE")
    fams = {}
    by_kernel = []
    for name in set(fetch) | set(write):
        fam = family(name)
        rd = 2.0 * fetch.get(name, (0.0, 0))[0] * 1024 / a.steps
        wr = write.get(name, (0.0, 0))[0] * 1024 / a.steps
        launches = max(fetch.get(name, (0, 0))[1], write.get(name, (0, 0))[1]) / a.steps
        by_kernel.append((rd + wr, rd, wr, launches, name))
        f = fams.setdefault(fam, {"read_bytes_per_step": 0.0, "write_bytes_per_step": 0.0, "launches_per_step": 0.0})
        f["read_bytes_per_step"] += rd
        f["write_bytes_per_step"] += wr
        f["launches_per_step"] += launches
    for f in fams.values():
        f["hbm_bytes_per_step"] = f["read_bytes_per_step"] + f["write_bytes_per_step"]
    if a.sq:
        # MFMA pipe busy: SQ_VALU_MFMA_BUSY_CYCLES counts SIMD-cycles an MFMA occupies (16 per
        # v_mfma_f32_16x16x32_f16, MI355X_MICROARCH.md cycle table), summed over all 1024 SIMDs; GRBM_GUI_ACTIVE is
        # the dispatch's GPU-busy cycles summed over the 8 XCDs.  busy = MFMA cycles / (GUI cycles / 8 * 1024)
        mb = load(a.sq, "SQ_VALU_MFMA_BUSY_CYCLES")
        gui = load(a.sq, "GRBM_GUI_ACTIVE")
        sqb = load(a.sq, "SQ_BUSY_CYCLES")
        acc = {}
        for name in set(mb) | set(gui):
            fam = family(name)
            m, g = acc.get(fam, (0.0, 0.0))
            acc[fam] = (m + mb.get(name, (0.0, 0))[0], g + gui.get(name, (0.0, 0))[0])
        for fam, (m, g) in acc.items():
            f = fams.setdefault(fam, {})
            f["mfma_busy_cycles_per_step"] = m / a.steps
            f["gui_active_cycles_per_step"] = g / 8.0 / a.steps
            f["mfma_busy"] = m / (g / 8.0 * 1024.0) if g > 0 else None
        per_kernel = []
        for name in mb:
            g = gui.get(name, (0.0, 0))[0]
            if g > 0:
                per_kernel.append((name, mb[name][0] / (g / 8.0 * 1024.0), g / 8.0 / a.steps, mb[name][1] / a.steps,
                                   sqb.get(name, (0.0, 0))[0] / a.steps))
        per_kernel.sort(key=lambda r: -r[2])
        top = [{"kernel": n[:120], "mfma_busy": round(b, 4), "gui_cycles_per_step": round(c), "launches_per_step": l,
                "sq_busy_cycles_per_step": round(q)} for n, b, c, l, q in per_kernel[:40]]
    out = {"label": a.label, "steps": a.steps,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950 "
                     "16-B/lane read calibration, MI355X_MICROARCH.md §HBM), KB -> bytes, summed per family / steps",
           "families": fams,
           "top_kernels_by_bytes": [{"kernel": n[:120], "hbm_bytes_per_step": round(t), "read": round(r),
                                     "write": round(w), "launches_per_step": round(l, 2)}
                                    for t, r, w, l, n in sorted(by_kernel, reverse=True)[:40]]}
    if a.sq:
        out["mfma_method"] = ("rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (own pass): "
                              "mfma_busy = MFMA SIMD-cycles / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)")
        out["top_kernels_by_cycles"] = top
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
