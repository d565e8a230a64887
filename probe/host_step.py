"""Is the captured config-4 step host-bound? (diagnostic, round 6)  The benched trainer is captured, then N steps are
issued back to back: the host time of the issuing loop (no synchronisation inside it) against the wall time once the
GPU has drained.  If the loop itself takes about as long as the wall time, the GPU waits for graph launches.
Also times one step's issue split by piece (torch.cuda.CUDAGraph.replay of each captured graph).  One JSON line."""
import json
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tf_depth_estimation_amd import _lib  # noqa: E402

args = types.SimpleNamespace(ddp="overlap", bucket_mb=256.0, sync_bn=False, net_overlap="on", adam_overlap="off",
                             deferred_adam="off", wgrad_overlap="on", wgrad_progs="auto", adam_bucket_mb=16.0,
                             exchange="auto", exchange_mode="segments")
_lib.check(_lib.load().tde_set_conv_math(4), "math")
tr, opts = bench.build_trainer(args, "config4", 8, 1, 0)
tr.capture()
for _ in range(10):
    tr.step()
torch.cuda.synchronize()
out = {"probe": "host issue time vs wall time of captured config-4 steps", "options": opts}
for n in (20, 50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        tr.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[f"n{n}"] = {"host_ms_per_step": round(1e3 * (t1 - t0) / n, 3), "wall_ms_per_step": round(1e3 * (t2 - t0) / n, 3)}
    print(n, out[f"n{n}"], flush=True)
# per graph: wrap every CUDAGraph.replay to time its host call during one step
orig = torch.cuda.CUDAGraph.replay
rec = []


def timed_replay(self):
    a = time.perf_counter()
    orig(self)
    rec.append((id(self), 1e3 * (time.perf_counter() - a)))


torch.cuda.CUDAGraph.replay = timed_replay
torch.cuda.synchronize()
t0 = time.perf_counter()
tr.step()
t1 = time.perf_counter()
torch.cuda.synchronize()
torch.cuda.CUDAGraph.replay = orig
out["one_step"] = {"host_ms": round(1e3 * (t1 - t0), 3), "replays_ms": [round(ms, 3) for _, ms in rec],
                   "replay_total_ms": round(sum(ms for _, ms in rec), 3)}
print(json.dumps(out))
