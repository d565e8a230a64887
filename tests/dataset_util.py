"""Synthetic on-disk dataset in the layout imageselect_Dataloader_optflow.py reads (test helper): <split>.txt
lines '<sub> <a> <b>', per sample <sub>/<a>_<b>.jpg (a tgt|src strip), <sub>/frame<a>_<b>.jpg_z.bin (raw
float32 depth), <sub>/<a>_<b>_cam.txt (9 comma-separated floats) and <sub>/<a>_<b>_tgt2src_proj.txt (33
space-separated floats + a trailing space: 34 fields, the last empty)."""
import os

import numpy as np


def _rigid(rng):
    """A random small rigid motion as a 4x4 matrix (Rodrigues of a random angle-axis, a unit-ish translation)."""
    ax = rng.standard_normal(3)
    ax /= np.linalg.norm(ax)
    th = rng.uniform(0.02, 0.2)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    T = np.eye(4)
    T[:3, :3] = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    T[:3, 3] = 0.1 * rng.standard_normal(3)
    return T


def make_dataset(root, n, strip_hw=(60, 180), image_hw=(30, 90), split="train", seed=0, sizes=None,
                 quality=92, rigid=False):
    """rigid=True: the two 4x4 matrices of each tgt2src_proj file are a rigid motion and its inverse (a camera
    pose the config-4 cam loss can take), else 32 random numbers."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    lines = []
    for k in range(n):
        sub = f"seq{k % 3}"
        os.makedirs(os.path.join(root, sub), exist_ok=True)
        a, b = f"{k:04d}", f"{(k * 7) % 13:02d}"
        fid = f"{a}_{b}"
        h, w = sizes[k] if sizes is not None else strip_hw
        # smooth texture + noise so the JPEG is not trivial
        yy, xx = np.mgrid[0:h, 0:w]
        img = np.stack([128 + 100 * np.sin(xx / (5.0 + c) + yy / (7.0 + 2 * c) + k) for c in range(3)], -1)
        img = np.clip(img + rng.normal(0, 12, img.shape), 0, 255).astype(np.uint8)
        Image.fromarray(img).save(os.path.join(root, sub, fid + ".jpg"), quality=quality)
        rng.uniform(0.5, 10.0, image_hw).astype("<f4").tofile(os.path.join(root, sub, "frame" + fid + ".jpg_z.bin"))
        fx, fy = rng.uniform(100, 300, 2)
        cam = [fx, 0.0, rng.uniform(40, 60), 0.0, fy, rng.uniform(10, 20), 0.0, 0.0, 1.0]
        with open(os.path.join(root, sub, fid + "_cam.txt"), "w") as f:
            f.write(",".join(f"{v:.6f}" for v in cam))
        if rigid:
            T = _rigid(rng)
            proj = list(T.reshape(-1)) + list(np.linalg.inv(T).reshape(-1)) + [rng.uniform(0.5, 2.0)]
        else:
            proj = list(rng.normal(0, 1, 32)) + [rng.uniform(0.5, 2.0)]
        with open(os.path.join(root, sub, fid + "_tgt2src_proj.txt"), "w") as f:
            f.write(" ".join(f"{v:.6f}" for v in proj) + " ")
        lines.append(f"{sub} {a} {b}\n")
    with open(os.path.join(root, f"{split}.txt"), "w") as f:
        f.writelines(lines)
    return root
