"""Upper bound of what a kernel family costs on the config-4 step's critical path (diagnostic, results garbage):
the benched step captured and replayed with every ABI call of the named families replaced by a no-op (or, for the
fused conv + BN forward, by the bare conv), timed like bench.py.  One eager step with the full library runs first, so
every buffer a skipped call would have written holds realistic values.

    SKIP=bnf,bnb python probe/skip_family.py [STEPS]

Families: bnf (BatchNorm forward: finalize + apply / one-kernel BN of the fused conv + BN calls), bnb (BatchNorm
backward), head (head fwd + bwd), warp (warp loss + pose prep/grad), pyr (depth/smooth loss pyramids), adam,
resize (nearest / bilinear), copy (copy_view)."""
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tf_depth_estimation_amd import _lib  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 100
SKIP = [s for s in os.environ.get("SKIP", "").split(",") if s]

lib = _lib.load()
args = types.SimpleNamespace(ddp="overlap", bucket_mb=32.0, sync_bn=False, net_overlap="on", adam_overlap="off",
                             deferred_adam="off", wgrad_overlap="on", wgrad_progs="auto", adam_bucket_mb=16.0)
_lib.check(lib.tde_set_conv_math(4), "math")
tr, _ = bench.build_trainer(args, "config4", 8, 1, 0)
tr.step_eager()
tr.flush()
torch.cuda.synchronize()


def noop(*a):
    return 0


FAMILIES = {
    "bnb": ["tde_bn_bwd"],
    "head": ["tde_head_fwd", "tde_head_bwd"],
    "warp": ["tde_warp_loss", "tde_warp_loss_multi", "tde_pose_prep", "tde_pose_prep_multi", "tde_pose_grad",
             "tde_pose_grad_spread", "tde_cam_loss"],
    "pyr": ["tde_loss_depth_pyramid", "tde_loss_depth_pyramid_multi", "tde_resize_area_fwd"],
    "adam": ["tde_adam_update"],
    "resize": ["tde_resize_nearest_fwd", "tde_resize_nearest_bwd", "tde_resize_bilinear_fwd",
               "tde_resize_bilinear_bwd"],
    "copy": ["tde_copy_view"],
}
for fam in SKIP:
    if fam == "bnf":
        cf, df = lib.tde_conv2d_fwd, lib.tde_deconv2d_fwd
        lib.tde_conv2d_fwd_bn = lambda d, x, w, z, bn, ws, wsb, st: cf(d, x, w, z, 0, ws, wsb, st)
        lib.tde_deconv2d_fwd_bn = lambda d, x, w, z, bn, ws, wsb, st: df(d, x, w, z, 0, ws, wsb, st)
        continue
    for name in FAMILIES[fam]:
        setattr(lib, name, noop)

tr.capture()
for _ in range(20):
    tr.step()
torch.cuda.synchronize()
best = None
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(STEPS):
        tr.step()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / STEPS
    best = ms if best is None else min(best, ms)
print(f"SKIP={','.join(SKIP) or '-'}: {best:.3f} ms/step ({8e3 / best:.0f} pairs/s)", flush=True)
tr.flush()
tr.release_graphs()
