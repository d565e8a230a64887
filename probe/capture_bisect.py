"""Diagnostic (round 3): which feature of the config-4 single-graph capture makes
hipStreamEndCapture segfault.  One capture + one replay per process, features chosen on the command line:
    python probe/capture_bisect.py [ov|ovs] [wg|wgp|wgs] [twin|solo] [B H W]
ov: depth_net's calls a forked branch (net overlap; ovs: disp_net's instead); wg: filter gradients of both
programs on side streams (forked branches; wgp / wgs: depth_net's / disp_net's only); solo: the non-twin (two
calls per net) step.  TDE_C4_INLINE_ADAM selects the per-net inline Adam."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_trainers import intrinsics, small_pose, texture  # noqa: E402
from tf_depth_estimation_amd import _api, train, variables  # noqa: E402

args = sys.argv[1:]
nums = [int(a) for a in args if a.isdigit()]
B, H, W = nums if len(nums) == 3 else (2, 64, 96)
variables.get_store().reset(seed=1)
_api.clear_programs()
tr = train.DepthThenCamTrainer(B, H, W, twin="solo" not in args)
lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(), torch.tensor(lab, dtype=torch.float32).cuda(),
             intrinsics(B, H, W).cuda(), small_pose(B, 4).cuda())
if "ovs" in args:
    tr.ov_net = "single"
if "wg" in args:
    tr.enable_wgrad_overlap(only=["single", "pair"])
elif "wgp" in args or "wgs" in args:
    tr.enable_wgrad_overlap(only=["pair"] if "wgp" in args else ["single"])
if "ov" in args or "ovs" in args:
    tr.enable_net_overlap()
print(f"[capture_bisect] {args} inline_adam={tr._inline_adam()} capturing", flush=True)
tr.capture(warmup=1, single_graph=True)
tr.step()
torch.cuda.synchronize()
print(f"[capture_bisect] {args} ok, graphs {len(tr.graphs)}, loss {tr.total_loss():.6f}", flush=True)
