"""Where the config-4 step's wall time goes, per stream (diagnostic): the benched trainer captured with a device stamp
after every op (program.StepTimeline), replayed, and each op's time taken as its stamp minus the previous stamp on
its stream (its kernels plus any cross-stream wait it started with).  Prints per-stream totals and the longest ops,
and writes the whole timeline (ops in stamp order with start offsets) to OUT.

    BRANCH=on|off python probe/step_timeline.py [OUT]"""
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tf_depth_estimation_amd import _lib  # noqa: E402
from tf_depth_estimation_amd.program import StepTimeline  # noqa: E402

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/timeline.txt"
args = types.SimpleNamespace(ddp="overlap", bucket_mb=32.0, sync_bn=False, net_overlap="on", adam_overlap="off",
                             deferred_adam="off", wgrad_overlap="on", wgrad_progs="auto", adam_bucket_mb=16.0,
                             exchange="auto", exchange_mode="graph")
_lib.check(_lib.load().tde_set_conv_math(4), "math")
tr, opts = bench.build_trainer(args, "config4", 8, 1, 0)


def timed(n=50):
    for _ in range(10):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        tr.step()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


tr.capture()
plain = timed()
tr.release_graphs()
tl = StepTimeline()
tr.set_timeline(tl)
tr.capture()
stamped = timed()
tr.step()
torch.cuda.synchronize()
iv = tl.intervals()
t0 = min(a for _, _, a, _ in iv)
names = {}
for label, sid, _, _ in iv:
    names.setdefault(sid, f"s{len(names)}<{label.split(':')[0]}>")
print(f"options {opts}; step {plain:.3f} ms plain, {stamped:.3f} ms with {len(tl.marks)} stamps; "
      f"stamped span {max(b for *_, b in iv) - t0:.1f} us")
for sid, nm in names.items():
    mine = [x for x in iv if x[1] == sid]
    print(f"{nm:40s} {len(mine):4d} ops  busy {sum(b - a for *_, a, b in mine):8.1f} us  "
          f"from {min(a for *_, a, _ in mine) - t0:8.1f} to {max(b for *_, b in mine) - t0:8.1f} us")
print("longest ops:")
for label, sid, a, b in sorted(iv, key=lambda x: x[2] - x[3])[:45]:
    print(f"  {b - a:7.1f} us  @{a - t0:8.1f}  {names[sid]:30s} {label}")
os.makedirs(os.path.dirname(OUT) or ".", exist_ok=True)
with open(OUT, "w") as f:
    f.write(f"# step {plain:.3f} ms plain, {stamped:.3f} ms stamped; options {opts}\n")
    for label, sid, a, b in sorted(iv, key=lambda x: x[3]):
        f.write(f"{a - t0:9.1f} {b - t0:9.1f} {b - a:8.1f}  {names[sid]:30s} {label}\n")
tr.release_graphs()
