"""Diagnostic (not collected by pytest): whole-gradient error of the config-4 step per conv math mode
and input seed, next to the oracle's own fp32 error -- the noise model behind check_grads_global.

    python tests/diag_grad_noise.py [TERM ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import losses as OL  # noqa: E402
from oracle import nets as ON  # noqa: E402
from test_gpu_nets import oracle_params_from  # noqa: E402
from test_gpu_trainers import C4_TERMS, intrinsics, small_pose, texture  # noqa: E402


def rel(g, r):
    return ((g - r).norm() / r.norm()).item()


def run(term, math, seed):
    from tf_depth_estimation_amd import _api, _lib, train, variables
    lib = _lib.load()
    _lib.check(lib.tde_set_conv_math(math))
    variables.get_store().reset(seed=1 + seed)
    _api.clear_programs()
    B, H, W = 2, 64, 96
    w = C4_TERMS[term] or dict(OL.W_CONFIG4)
    tr = train.DepthThenCamTrainer(B, H, W, weights=w)
    il, ir = texture(B, H, W, 1 + 10 * seed), texture(B, H, W, 2 + 10 * seed)
    g = np.random.default_rng(3 + seed)
    lab = g.uniform(0.1, 2.0, (B, H, W, 1))
    lab[g.uniform(size=lab.shape) < 0.05] = np.nan
    lab = torch.tensor(lab, dtype=torch.float32)
    K = intrinsics(B, H, W)
    gt = small_pose(B, 4 + seed)
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), gt.cuda())
    chunks = [tr.single.chunk, tr.pair.chunk]
    out = {}
    for dt in (torch.float64, torch.float32):
        Pss, Ppp = oracle_params_from(chunks[0], "", dt), oracle_params_from(chunks[1], "", dt)
        x = {k: v.to(dt) for k, v in dict(il=il, ir=ir).items()}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        total, _ = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.to(dt),
                                             K.to(dt), gt.to(dt), w=w)
        total.backward()
        out[dt] = {k: v.grad for P in (Pss, Ppp) for k, v in P.vars.items()}
    names = sorted(out[torch.float64])
    r = torch.cat([out[torch.float64][n].reshape(-1) for n in names])
    c = torch.cat([out[torch.float32][n].double().reshape(-1) for n in names])
    res = []
    for rep in range(2):
        tr.phase_compute()
        torch.cuda.synchronize()
        gpu = {}
        for ch in chunks:
            gpu.update({k: ch.grad_view(k) for k in ch.names()})
        gv = torch.cat([gpu[n].detach().double().cpu().reshape(-1) for n in names])
        res.append(rel(gv, r))
    return res, rel(c, r)


if __name__ == "__main__":
    terms = sys.argv[1:] or ["depth_l1", "all"]
    for term in terms:
        for seed in range(3):
            for math in (0, 3):
                eg, ec = run(term, math, seed)
                print(f"{term:9s} seed {seed} math {math}: gpu {eg[0]:.2e} {eg[1]:.2e}  cpu32 {ec:.2e}  "
                      f"ratio {max(eg) / ec:.2f}", flush=True)
