"""Per-layer HIP-event timing of one training step (diagnostic; not part of the bench contract).

    python scripts/layer_profile.py [--workload config2] [--batch 8]
Prints, per (kernel family, layer): time, algorithmic TFLOP/s and the GEMM shape."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from tf_depth_estimation_amd.program import KernelTimer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config2")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--loss-vs", type=float, default=0.0,
                    help="also rank conv entries by ms lost against this TFLOP/s reference")
    ap.add_argument("--math", default="fp32")
    a = ap.parse_args()
    from tf_depth_estimation_amd import _lib
    _lib.check(_lib.load().tde_set_conv_math(_lib.CONV_MATH[a.math]), "conv math")
    N = a.batch or bench.WORKLOADS[a.workload][2]
    tr = bench.make_trainer(a.workload, N)
    tr.set_batch(*[t.cuda() for t in bench.make_batch(a.workload, N, 0)])
    progs = [p for p in (getattr(tr, "prog", None), getattr(tr, "single", None), getattr(tr, "pair", None)) if p]
    tr.step_eager()
    tr.step_eager()
    timer = KernelTimer()
    for p in progs:
        p.timer = timer
    tr.step_eager()
    for p in progs:
        p.timer = None
    rows = timer.by_tag()
    agg = {}
    for fam, tag, ms, fl in rows:
        k = (fam, tag)
        t, f, n = agg.get(k, (0.0, 0.0, 0))
        agg[k] = (t + ms, f + fl, n + 1)
    tot = sum(v[0] for v in agg.values())
    print(f"total instrumented ms {tot:.3f}")
    for (fam, tag), (ms, fl, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 and fl > 0 else 0.0
        print(f"{ms:8.3f} ms {100 * ms / tot:5.1f}%  {fam:11s} {tag:28s} x{n}  {tf:7.2f} TF/s  {fl / 1e9:7.2f} GF")
    if a.loss_vs > 0:
        ref = a.loss_vs * 1e12
        rows = [(ms - fl / ref * 1e3, ms, fam, tag, fl) for (fam, tag), (ms, fl, n) in agg.items()
                if fam.startswith("conv")]
        print(f"\nconv ms lost vs {a.loss_vs} TF/s: total {sum(r[0] for r in rows):.3f} ms")
        for lost, ms, fam, tag, fl in sorted(rows, reverse=True)[:a.top]:
            print(f"{lost:8.3f} lost {ms:8.3f} ms  {fam:11s} {tag:20s} {fl / (ms * 1e-3) / 1e12:7.2f} TF/s")


if __name__ == "__main__":
    main()
