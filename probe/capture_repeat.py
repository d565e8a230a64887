"""Diagnostic (round 3): capture the config-4 step with the net overlap as ONE graph (depth_net's
calls a forked capture branch; filter gradients on their own side streams) again and again in one process -- the
round-2 crash came after ~40 captures -- and replay each once.  Every side / capture stream is now a dedicated HIP
stream (_lib.owned_stream); torch's pooled torch.cuda.Stream() could hand a "new" side stream that aliases the
capture stream, turning a fork / join into a self-wait.
    python probe/capture_repeat.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_trainers import intrinsics, small_pose, texture  # noqa: E402
from tf_depth_estimation_amd import _api, train, variables  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
B, H, W = 2, 64, 96
lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
losses = []
for i in range(n):
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    tr = train.DepthThenCamTrainer(B, H, W)
    tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(), torch.tensor(lab, dtype=torch.float32).cuda(),
                 intrinsics(B, H, W).cuda(), small_pose(B, 4).cuda())
    tr.enable_wgrad_overlap()
    tr.enable_net_overlap()
    tr.capture(warmup=1, single_graph=True)
    assert len(tr.graphs) == 1 and tr.ov_seq is None
    tr.step()
    torch.cuda.synchronize()
    losses.append(tr.total_loss())
    print(f"[capture_repeat] {i + 1}/{n} captures ok, loss {losses[-1]:.6f}", flush=True)
    del tr
print("[capture_repeat] all", n, "single-graph captures replayed", flush=True)
