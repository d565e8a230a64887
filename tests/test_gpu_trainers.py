"""Step-level GPU parity of the warp-loss configs (3, 4, 5) against the float64 oracle loss loops
(oracle/losses.py).  Same criteria as tests/test_gpu_nets.py: loss value to 1e-5 relative, every
parameter gradient within max(1e-3, 4 x the fp32-oracle's own error)."""
import numpy as np
import pytest
import torch

from oracle import geometry as OG
from oracle import losses as OL
from oracle import nets as ON

from test_gpu_nets import check_grads, oracle_params_from

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def fresh_store():
    from tf_depth_estimation_amd import _api, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    yield


def texture(B, H, W, seed):
    """SURVEY.md §8(d) config 4 images: sum of 8 random sinusoids + 0.02 N(0,1), clipped to +-0.5."""
    g = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    out = np.zeros((B, H, W, 3))
    for b in range(B):
        for c in range(3):
            acc = np.zeros((H, W))
            for _ in range(8):
                fx, fy = g.uniform(0.02, 0.25, 2)
                acc += g.uniform(0.05, 0.15) * np.sin(fx * xx + fy * yy + g.uniform(0, 6.28))
            out[b, :, :, c] = acc
    out += 0.02 * g.standard_normal(out.shape)
    return torch.tensor(np.clip(out, -0.5, 0.5), dtype=torch.float32)


def intrinsics(B, H, W):
    fx, fy, cx, cy = 0.89 * W, 1.19 * H, 0.5 * W, 0.5 * H
    K = torch.tensor([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], dtype=torch.float64).expand(B, 3, 3)
    return OG.get_multi_scale_intrinsics(K, 4).float()


def small_pose(B, seed):
    g = np.random.default_rng(seed)
    t = g.standard_normal((B, 3))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    ax = g.standard_normal((B, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    r = ax * g.uniform(0.02, 0.2, (B, 1))
    return torch.tensor(np.concatenate([t * 0.1, r], 1), dtype=torch.float32)


def test_config4_depth_then_cam_step():
    from tf_depth_estimation_amd import train
    B, H, W = 2, 64, 96
    tr = train.DepthThenCamTrainer(B, H, W)
    il, ir = texture(B, H, W, 1), texture(B, H, W, 2)
    g = np.random.default_rng(3)
    lab = g.uniform(0.1, 2.0, (B, H, W, 1))
    lab[g.uniform(size=lab.shape) < 0.05] = np.nan
    lab = torch.tensor(lab, dtype=torch.float32)
    K = intrinsics(B, H, W)
    gt = small_pose(B, 4)
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), gt.cuda())
    chunks = {"s": tr.single.chunk, "p": tr.pair.chunk}
    Ps = {dt: (oracle_params_from(chunks["s"], "", dt), oracle_params_from(chunks["p"], "", dt))
          for dt in (torch.float64, torch.float32)}
    tr.phase_compute()
    torch.cuda.synchronize()
    parts = tr.loss_parts()
    grads = {}
    for dt, (Pss, Ppp) in Ps.items():
        x = {k: v.to(dt) for k, v in dict(il=il, ir=ir).items()}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        total, rparts = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.to(dt),
                                                  K.to(dt), gt.to(dt))
        total.backward()
        if dt == torch.float64:
            for k in ("smooth", "depth", "exp", "cam"):
                assert abs(parts[k] - rparts[k].item()) <= 1e-5 * abs(rparts[k].item()) + 1e-9, k
            assert abs(parts["photo"] - rparts["pixel"].item()) <= 1e-5 * rparts["pixel"].item()
            assert abs(parts["consist"] - rparts["consist"].item()) <= 1e-4 * rparts["consist"].item()
        grads[dt] = {k: v.grad for P in (Pss, Ppp) for k, v in P.vars.items()}
    gpu = {}
    for c in chunks.values():
        gpu.update({k: c.grad_view(k) for k in c.names()})
    check_grads(gpu, grads[torch.float64], grads[torch.float32])


def test_config3_optflow_combine_step():
    from tf_depth_estimation_amd import train
    B, H, W = 2, 64, 96
    tr = train.OptflowCombineTrainer(B, H, W)
    il, ir = texture(B, H, W, 5), texture(B, H, W, 6)
    lab = torch.tensor(np.random.default_rng(7).uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32)
    K = intrinsics(B, H, W)
    T = OG.pose_vec2mat(small_pose(B, 8).double(), "angleaxis").float()
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), T.cuda())
    grads = {}
    Ps = {dt: oracle_params_from(tr.prog.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    tr.phase_compute()
    torch.cuda.synchronize()
    for dt, P in Ps.items():
        outs = ON.disp_net_depthflow(P, torch.cat([il, ir], -1).to(dt), True, scope="model/depth_net")
        total, _ = OL.loss_optflow_combine(outs, il.to(dt), ir.to(dt), lab.to(dt), K.to(dt), T.to(dt))
        total.backward()
        if dt == torch.float64:
            assert abs(tr.total_loss() - total.item()) <= 1e-5 * total.item()
        grads[dt] = {k: v.grad for k, v in P.vars.items()}
    check_grads({k: tr.prog.chunk.grad_view(k) for k in tr.prog.chunk.names()}, grads[torch.float64],
                grads[torch.float32])


def test_config5_refine_step():
    from tf_depth_estimation_amd import train
    B, H, W = 2, 64, 96
    tr = train.RefineTrainer(B, H, W)
    x1, x2 = texture(B, H, W, 9), texture(B, H, W, 10)
    gt = torch.tensor(np.random.default_rng(11).uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32)
    K = intrinsics(B, H, W)
    T = OG.pose_vec2mat(small_pose(B, 12).double(), "angleaxis").float()
    tr.set_batch(x1.cuda(), x2.cuda(), gt.cuda(), K.cuda(), T.cuda())
    Ps = {dt: oracle_params_from(tr.prog.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    tr.phase_compute()
    torch.cuda.synchronize()
    grads = {}
    for dt, P in Ps.items():
        d = ON.disp_net(P, x1.to(dt), True, scope="model/depth_net")
        total, _ = OL.loss_refine(d, x1.to(dt), x2.to(dt), gt.to(dt), T.to(dt), K.to(dt))
        total.backward()
        if dt == torch.float64:
            assert abs(tr.total_loss() - total.item()) <= 1e-5 * total.item()
        grads[dt] = {k: v.grad for k, v in P.vars.items()}
    check_grads({k: tr.prog.chunk.grad_view(k) for k in tr.prog.chunk.names()}, grads[torch.float64],
                grads[torch.float32])


def test_warp_fwd_matches_oracle():
    """Forward-only projective_inverse_warp kernel vs utils_lr semantics (coords, wmask, z, samples)."""
    from tf_depth_estimation_amd import _lib
    from tf_depth_estimation_amd._lib import ptr
    B, H, W = 2, 24, 32
    img = texture(B, H, W, 13)
    depth = torch.tensor(np.random.default_rng(14).uniform(0.5, 3.0, (B, H, W)), dtype=torch.float32)
    K = intrinsics(B, H, W)[:, 0].contiguous()
    pose = small_pose(B, 15)
    gK, gpose, gimg, gdep = K.cuda().reshape(B, 9).contiguous(), pose.cuda(), img.cuda(), depth.cuda()
    P, Kinv, T = (torch.empty(B, n, device="cuda") for n in (12, 9, 16))
    lib, st = _lib.load(), _lib.stream_ptr()
    _lib.check(lib.tde_pose_prep(B, ptr(gpose), None, ptr(gK), ptr(T), ptr(P), ptr(Kinv), st))
    out, coords, wm, z = (torch.empty(B, H, W, c, device="cuda") for c in (3, 2, 1, 1))
    _lib.check(lib.tde_warp_fwd(B, H, W, 3, ptr(gdep), 0, ptr(P), ptr(Kinv), None, ptr(gimg), H, W, ptr(out),
                                ptr(coords), None, None, ptr(wm), ptr(z), st))
    ro, rc, rw, rz, rT = OG.projective_inverse_warp(img.double(), depth.double(), pose.double(), K.double())
    torch.cuda.synchronize()
    assert (T.cpu().reshape(B, 4, 4).double() - rT).abs().max() < 1e-5
    assert (coords.cpu().double() - rc).abs().max() < 1e-3
    assert (z.cpu().double() - rz).abs().max() < 1e-4
    assert (out.cpu().double() - ro).abs().max() < 1e-4
    assert (wm.cpu().double() - rw).abs().max() < 1e-4
