"""Host cost of replaying the config-4 step's graphs (diagnostic): is the step bound by the GPU or by the host
submitting graph nodes?  For the benched trainer (BRANCH=on|off): the GPU step time (back-to-back replays), the host
time of one step() issued onto an idle GPU (the call's own duration) and its wall time to completion, and per piece
graph its host replay() time."""
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tf_depth_estimation_amd import _lib  # noqa: E402

args = types.SimpleNamespace(ddp="overlap", bucket_mb=32.0, sync_bn=False, net_overlap="on", adam_overlap="off",
                             deferred_adam="off", wgrad_overlap="on", wgrad_progs="auto", adam_bucket_mb=16.0,
                             exchange="auto", exchange_mode="graph")
_lib.check(_lib.load().tde_set_conv_math(4), "math")
tr, opts = bench.build_trainer(args, os.environ.get("WORKLOAD", "config4"), 8, 1, 0)
tr.capture()
for _ in range(10):
    tr.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    tr.step()
torch.cuda.synchronize()
gpu = 1e3 * (time.perf_counter() - t0) / 50
host, wall = [], []
for _ in range(20):
    torch.cuda.synchronize()
    a = time.perf_counter()
    tr.step()
    b = time.perf_counter()
    torch.cuda.synchronize()
    c = time.perf_counter()
    host.append(1e3 * (b - a))
    wall.append(1e3 * (c - a))
host.sort()
wall.sort()
print(f"{os.environ.get('WORKLOAD', 'config4')} options {opts}: back-to-back {gpu:.3f} ms/step; one step onto an idle "
      f"GPU: host call {host[10]:.3f} ms, wall {wall[10]:.3f} ms (medians)")
seq = getattr(tr, "ov_seq", None)
graphs = []
if seq:
    for where, segs in seq:
        for g, _ in (segs or []):
            if g is not None:
                graphs.append((where, g))
else:
    graphs = [("step", g) for g in tr.graphs]
for where, g in graphs:
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        g.replay()
        ts.append(1e3 * (time.perf_counter() - a))
        torch.cuda.synchronize()
    ts.sort()
    print(f"  graph [{where:5s}]: host replay() {ts[2]:.3f} ms")
tr.release_graphs()
