"""Generate the committed golden vectors under tests/golden/ (TEST INFRASTRUCTURE).

The reference ships no fixtures, golden outputs or tests, and TensorFlow 1.x is not installable here
(SURVEY.md §8c), so these vectors come from the float64 oracle restatement (oracle/), which is itself
pinned by the known-answer tests in tests/test_oracle_kat.py.  They freeze the oracle's answers so
that (a) the CPU suite detects any drift of the oracle, and (b) the GPU suite checks the HIP path
against stored numbers, independently of the oracle code that runs beside it.

Every input is reproducible from the seeds stored next to it: images are numpy PCG64 draws, weights
are slim's Glorot-uniform drawn per variable from PCG64([seed, crc32(name)]) and rounded to fp32
(exactly what the product's variable store holds), BN beta 0, moving mean 0 / variance 1.

  config1_fwd.npz   BASELINE configs[0]: nets_depth.disp_net (nets_depth.py:76-199) on one 128x96 pair,
                    is_training True and False -> the 8 outputs of nets_depth.py:199 (fp32-rounded)
  warp.npz          projective_inverse_warp (utils_lr.py:222-256) on a 2x12x16 batch with explicit
                    inputs, pose formats 'angleaxis' and 'eular' (pose_vec2mat, utils_lr.py:106-149)
  losses.npz        compute_smooth_loss (train_depth_then_cam_lr.py:59-68) and the config-2 loss
                    (train_depth_only.py:162-219) on explicit small inputs

Run:  python tests/golden/make_golden.py   (CPU, ~10 s)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import geometry as G  # noqa: E402
from oracle import losses as OL  # noqa: E402
from oracle import nets as ON  # noqa: E402

CONFIG1 = dict(N=1, H=96, W=128, C=6, x_seed=0, w_seed=1, scope="model/depth_net")


def config1_input():
    g = np.random.default_rng(CONFIG1["x_seed"])
    return g.uniform(-0.5, 0.5, size=(CONFIG1["N"], CONFIG1["H"], CONFIG1["W"], CONFIG1["C"])).astype(np.float32)


def fp32_params(seed):
    """Oracle params holding the fp32-rounded Glorot draws (the product's stored values)."""
    P = ON.Params(seed=seed)
    get = P.get

    def get32(name, shape, init):
        if name not in P.vars:
            t = get(name, shape, init)
            P.vars[name] = t.detach().float().double().requires_grad_(True)
        return P.vars[name]
    P.get = get32
    return P


def config1_outputs(is_training):
    x = torch.tensor(config1_input(), dtype=torch.float64)
    P = fp32_params(CONFIG1["w_seed"])
    with torch.no_grad():
        outs = ON.disp_net_depthflow(P, x, is_training, scope=CONFIG1["scope"])
    return [o.numpy() for o in outs]


def warp_case():
    g = np.random.default_rng(11)
    B, H, W = 2, 12, 16
    img = g.uniform(-0.5, 0.5, (B, H, W, 3)).astype(np.float32)
    depth = g.uniform(1.0, 4.0, (B, H, W)).astype(np.float32)
    t = g.normal(0, 0.2, (B, 3))
    ax = g.normal(0, 1, (B, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    r = ax * g.uniform(0.02, 0.2, (B, 1))
    pose = np.concatenate([t, r], 1).astype(np.float32)
    K = np.zeros((B, 3, 3), np.float32)
    K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2], K[:, 2, 2] = 0.89 * W, 1.19 * H, 0.5 * W, 0.5 * H, 1.0
    d = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    out, coords, wmask, z, pose4 = G.projective_inverse_warp(d(img), d(depth), d(pose), d(K), "angleaxis")
    eo, ec, ew, ez, ep = G.projective_inverse_warp(d(img), d(depth), d(pose), d(K), "eular")
    return dict(img=img, depth=depth, pose=pose, K=K, warped=out.numpy(), coords=coords.numpy(),
                wmask=wmask.numpy(), z=z.numpy(), pose4=pose4.numpy(),
                e_warped=eo.numpy(), e_coords=ec.numpy(), e_wmask=ew.numpy(), e_z=ez.numpy(), e_pose4=ep.numpy())


def loss_case():
    g = np.random.default_rng(21)
    N, H, W = 2, 32, 48
    disps = [g.uniform(0.2, 3.0, (N, H >> s, W >> s, 1)).astype(np.float32) for s in range(4)]
    label = g.uniform(0.25, 4.0, (N, H, W, 1)).astype(np.float32)
    d = [torch.tensor(a, dtype=torch.float64) for a in disps]
    total, parts = OL.loss_depth_only(d, torch.tensor(label, dtype=torch.float64))
    out = {f"disp{s}": disps[s] for s in range(4)}
    out.update(label=label, total=np.float64(total.item()), smooth=np.float64(parts["smooth"].item()),
               depth=np.float64(parts["depth"].item()),
               smooth0=np.float64(OL.compute_smooth_loss(d[0]).item()),
               smooth0_recip=np.float64(OL.compute_smooth_loss(1.0 / d[0]).item()))
    return out


def generate():
    arrays = {"x": config1_input()}
    for mode, tr in (("train", True), ("infer", False)):
        for i, o in enumerate(config1_outputs(tr)):
            arrays[f"{mode}_{i}"] = o.astype(np.float32)
    return {"config1_fwd.npz": arrays, "warp.npz": warp_case(), "losses.npz": loss_case()}


def main():
    for name, arrays in generate().items():
        np.savez_compressed(os.path.join(HERE, name), **arrays)
        print(name, {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
