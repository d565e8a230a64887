"""Diagnostic: capture the config-4 step with the net overlap (small shapes) and replay it once."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_trainers import texture, intrinsics, small_pose
from tf_depth_estimation_amd import _api, train, variables

variables.get_store().reset(seed=1)
_api.clear_programs()
B, H, W = 2, 64, 96
tr = train.DepthThenCamTrainer(B, H, W)
lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(), torch.tensor(lab, dtype=torch.float32).cuda(),
             intrinsics(B, H, W).cuda(), small_pose(B, 4).cuda())
if len(sys.argv) > 1 and sys.argv[1] == "wgrad":
    tr.enable_wgrad_overlap()
tr.enable_net_overlap()
print("capturing", flush=True)
tr.capture(warmup=1)
print("captured", flush=True)
tr.step()
torch.cuda.synchronize()
print("replayed", tr.total_loss(), flush=True)
