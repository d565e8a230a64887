"""Step-level GPU parity of the warp-loss configs (3, 4, 5) against the float64 oracle loss loops
(oracle/losses.py).  Same criteria as tests/test_gpu_nets.py: loss value to 1e-5 relative, every
parameter gradient within max(1e-3, 4 x the fp32-oracle's own error)."""
import numpy as np
import pytest
import torch

from oracle import geometry as OG
from oracle import losses as OL
from oracle import nets as ON

from test_gpu_nets import GRAD_FACTOR, check_grads, check_grads_global, oracle_params_from

# an empty captured segment is dropped, not replayed (train._end_segment): the warning must not surface
pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("error:The CUDA Graph is empty")]


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


C4_TERMS = {
    "smooth": dict(smooth=1.0, data=0.0, depth=0.0, exp=0.0, cam=0.0),
    "depth_l1": dict(smooth=0.0, data=0.0, depth=20.0, exp=0.0, cam=0.0),   # also scales consist
    "photo_exp": dict(smooth=0.0, data=10.0, depth=0.0, exp=1.0, cam=0.0),
    "cam": dict(smooth=0.0, data=0.0, depth=0.0, exp=0.0, cam=5.0),
    "all": None,
}


@pytest.fixture(params=[0, 3, 4], ids=["fp32", "bf16x6r", "fp16x3"])
def step_math(request):
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    prev = lib.tde_get_conv_math()
    _lib.check(lib.tde_set_conv_math(request.param))
    yield request.param
    _lib.check(lib.tde_set_conv_math(prev))


@pytest.mark.parametrize("term,twin", [(t, True) for t in C4_TERMS] + [("all", False)])
def test_config4_depth_then_cam_step(term, twin, step_math):
    """twin=True (default): each net's two calls as one row-grouped batch-2B call (grouped BatchNorm);
    twin=False: the four separate calls.  Both against the oracle's four separate calls."""
    from tf_depth_estimation_amd import train
    B, H, W = 2, 64, 96
    w = C4_TERMS[term] or dict(OL.W_CONFIG4)
    tr = train.DepthThenCamTrainer(B, H, W, weights=w, twin=twin)
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
                                                  K.to(dt), gt.to(dt), w=w)
        total.backward()
        if dt == torch.float64:
            def val(t):
                return t.item() if torch.is_tensor(t) else float(t)
            for k in ("smooth", "depth", "exp", "cam"):
                assert abs(parts[k] - val(rparts[k])) <= 1e-5 * abs(val(rparts[k])) + 1e-9, k
            assert abs(parts["photo"] - val(rparts["pixel"])) <= 1e-5 * val(rparts["pixel"]) + 1e-9
            assert abs(parts["consist"] - val(rparts["consist"])) <= 1e-4 * val(rparts["consist"]) + 1e-9
        grads[dt] = {k: v.grad for P in (Pss, Ppp) for k, v in P.vars.items()}
    gpu = {}
    for c in chunks.values():
        gpu.update({k: c.grad_view(k) for k in c.names()})
    # 1/disp smoothness of near-flat random-init disparities is sign-noise in fp32 (see module doc of
    # test_gpu_nets); the per-kernel gradient checks are in test_warp_loss_kernel_gradients, here the
    # whole gradient vector is compared.
    check_grads_global(gpu, grads[torch.float64], grads[torch.float32], GRAD_FACTOR[step_math])


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
    # whole-gradient criterion (like config 4): per tensor, training-mode BN backward leaves even the
    # oracle's own fp32 gradients 5-9% off fp64 on some deep tensors, too noisy for a per-tensor bar
    check_grads_global({k: tr.prog.chunk.grad_view(k) for k in tr.prog.chunk.names()}, grads[torch.float64],
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
    check_grads_global({k: tr.prog.chunk.grad_view(k) for k in tr.prog.chunk.names()}, grads[torch.float64],
                grads[torch.float32])


@pytest.mark.parametrize("with_logits", [True, False])
def test_warp_loss_kernel_gradients(with_logits):
    """tde_warp_loss + tde_pose_grad on well-conditioned random inputs vs float64 autograd of the
    oracle (utils_lr.projective_inverse_warp / consistent_depth_loss, train_depth_then_cam_lr.py:253-340):
    loss parts and d/d(disp, logits, disp_other, pose vector)."""
    from tf_depth_estimation_amd import _lib, losses as Ls
    from tf_depth_estimation_amd._lib import ptr
    B, H, W = 2, 24, 32
    g = np.random.default_rng(21)
    src, tgt = texture(B, H, W, 22), texture(B, H, W, 23)
    disp = torch.tensor(g.uniform(0.3, 1.0, (B, H, W, 1)), dtype=torch.float32)
    disp_o = torch.tensor(g.uniform(0.3, 1.0, (B, H, W, 1)), dtype=torch.float32)
    logits = torch.tensor(g.standard_normal((B, H, W, 2)), dtype=torch.float32)
    pose = small_pose(B, 24)
    K = intrinsics(B, H, W)[:, 0].contiguous()
    pw, ew, cw = 10.0, 1.0, 20.0
    # GPU
    d = {k: v.cuda().contiguous() for k, v in dict(src=src, tgt=tgt, disp=disp, disp_o=disp_o, logits=logits,
                                                    pose=pose, K=K.reshape(B, 9)).items()}
    P, Kinv, T = (torch.empty(B, n, device="cuda") for n in (12, 9, 16))
    Ls.pose_prep(d["K"], T=T, P=P, Kinv=Kinv, vec=d["pose"])
    acc = torch.zeros(3, dtype=torch.float64, device="cuda")
    gd, gdo, gl = (torch.zeros_like(d[k]) for k in ("disp", "disp_o", "logits"))
    gP = torch.zeros(1, B, 12, dtype=torch.float64, device="cuda")
    Ls.warp_loss(acc, 0, d["src"], d["tgt"], P=P, Kinv=Kinv, disp=d["disp"],
                 logits=d["logits"] if with_logits else None, disp_other=d["disp_o"] if with_logits else None,
                 photo_w=pw, exp_w=ew, consist_w=cw, g_disp=gd, g_logits=gl if with_logits else None,
                 g_other=gdo if with_logits else None, g_P=gP)
    gpose = torch.zeros(B, 6, device="cuda")
    lib = _lib.load()
    _lib.check(lib.tde_pose_grad(B, 1, ptr(d["pose"]), ptr(d["K"]), 9, ptr(gP), None, ptr(gpose), 0,
                                 _lib.stream_ptr()))
    torch.cuda.synchronize()
    # oracle (float64 autograd)
    r = {k: v.double().clone().requires_grad_(True) for k, v in dict(disp=disp, disp_o=disp_o, logits=logits,
                                                                     pose=pose).items()}
    out, coords, _, z, _ = OG.projective_inverse_warp(src.double(), (1.0 / r["disp"])[..., 0], r["pose"], K.double())
    err = (out - tgt.double()).abs()
    if with_logits:
        p1 = torch.softmax(r["logits"], -1)[..., 1:2]
        ref = torch.zeros(B, H, W, 2, dtype=torch.float64)
        ref[..., 1] = 1
        photo = (err * p1).mean() * pw
        exp = ew * (-(ref * torch.log_softmax(r["logits"], -1)).sum(-1)).mean()
        cons = (OG.consistent_depth_loss(1.0 / r["disp_o"], z, coords) * p1).mean() * cw
    else:
        photo, exp, cons = err.mean() * pw, torch.zeros(()), torch.zeros(())
    (photo + exp + cons).backward()
    got = acc.cpu().tolist()
    for a_, b_ in zip(got, (photo.item(), exp.item(), cons.item())):
        assert abs(a_ - b_) <= 1e-5 * abs(b_) + 1e-9
    from test_gpu_nets import rel_err
    assert rel_err(gd, r["disp"].grad) <= 1e-3
    assert rel_err(gpose, r["pose"].grad) <= 1e-3
    if with_logits:
        assert rel_err(gl, r["logits"].grad) <= 1e-4
        assert rel_err(gdo, r["disp_o"].grad) <= 1e-3


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


@pytest.mark.parametrize("where", ["side", "wgrad"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
@pytest.mark.parametrize("cfg", ["config2", "config4"])
def test_adam_overlap_matches_plain(cfg, graph, where):
    """Bucketed Adam on a side stream during backward (Trainer.enable_adam_overlap; a graph branch under
    capture) updates every element as the single Adam launch after backward: parameters and moments
    bit-identical.  Config 2 after three steps; config 4 (shared-variable nets: a bucket is final only at
    its net's second backward call) after one step with every loss term on (depth / consistency weight 20) in
    the deterministic warp-loss mode (Trainer.enable_deterministic: fixed-point scatter, fixed-order block sums;
    two plain runs are checked to agree bit for bit first).  With float atomics, run-to-run rounding makes
    Adam's first update flip sign on near-zero gradients, which no tolerance separates from a wrong bucket.
    where="wgrad": the buckets run on the programs' filter-gradient streams (enable_wgrad_overlap), against
    the same split backward run serially with the single Adam launch after it."""
    from tf_depth_estimation_amd import _api, train, variables
    steps = 3 if cfg == "config2" else 1

    def run(overlap):
        variables.get_store().reset(seed=1)
        _api.clear_programs()
        B, H, W = 2, 64, 96
        if cfg == "config2":
            tr = train.DepthOnlyTrainer(B, H, W)
            g = np.random.default_rng(9)
            tr.set_batch(torch.tensor(g.uniform(-0.5, 0.5, (B, H, W, 3)), dtype=torch.float32).cuda(),
                         torch.tensor(g.uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32).cuda())
        else:
            tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
            lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
            tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                         torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(),
                         small_pose(B, 4).cuda())
        if where == "wgrad":
            tr.enable_wgrad_overlap(serial=not overlap)
        if overlap:
            ov = tr.enable_adam_overlap(bucket_mb=0.5, on_wgrad_stream=(where == "wgrad"))
            assert len(ov.buckets) > 4
        if graph:
            tr.capture(warmup=1)
        for _ in range(steps):
            tr.step()
        torch.cuda.synchronize()
        if overlap and not graph:
            assert len(ov.done) == len(ov.buckets)
        return [(c.flat.clone(), c.adam_m.clone(), c.adam_v.clone()) for c in tr.chunks]

    ref = run(False)
    if cfg == "config4":
        for a, b in zip(ref, run(False)):
            assert all(torch.equal(x, y) for x, y in zip(a, b)), "plain config-4 step not deterministic"
    for (pa, ma, va), (pb, mb, vb) in zip(ref, run(True)):
        assert torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb)


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
@pytest.mark.parametrize("cfg", ["config2", "config4"])
def test_wgrad_overlap_matches_serial(cfg, graph):
    """Filter gradients on a side stream (Trainer.enable_wgrad_overlap; a parallel graph branch under
    capture, joined at the end of backward; the BN backward alternates two dz buffers and waits for the
    filter gradient that last read the one it overwrites) against the same split calls serially on one
    stream: bit-identical.  Config 2 after three steps; config 4 (two backward calls per shared-variable
    chunk, accumulating on the side stream; two programs, two side streams) after one step with all loss
    terms in the deterministic warp-loss mode (checked: two serial runs agree bit for bit first)."""
    from tf_depth_estimation_amd import _api, train, variables
    steps = 3 if cfg == "config2" else 1

    def run(mode):
        variables.get_store().reset(seed=1)
        _api.clear_programs()
        B, H, W = 2, 64, 96
        if cfg == "config2":
            tr = train.DepthOnlyTrainer(B, H, W)
            g = np.random.default_rng(9)
            tr.set_batch(torch.tensor(g.uniform(-0.5, 0.5, (B, H, W, 3)), dtype=torch.float32).cuda(),
                         torch.tensor(g.uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32).cuda())
        else:
            tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
            lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
            tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                         torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(),
                         small_pose(B, 4).cuda())
        tr.enable_wgrad_overlap(serial=(mode == "serial"))
        if graph:
            tr.capture(warmup=1)
        p0 = [c.flat.clone() for c in tr.chunks]
        for _ in range(steps):
            tr.step()
        torch.cuda.synchronize()
        return [(c.flat.clone(), c.grad.clone(), c.flat - q) for c, q in zip(tr.chunks, p0)]

    ref = run("serial")
    if cfg == "config4":
        for (pa, ga, _), (pb, gb, _) in zip(ref, run("serial")):
            assert torch.equal(ga, gb) and torch.equal(pa, pb), "serial config-4 step not deterministic"
    for (pa, ga, _), (pb, gb, _) in zip(ref, run("overlap")):
        assert torch.equal(ga, gb) and torch.equal(pa, pb)


@pytest.mark.parametrize("mid_flush", [False, True], ids=["end_flush", "mid_flush"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
@pytest.mark.parametrize("cfg", ["config2", "config4"])
def test_deferred_adam_matches_plain(cfg, graph, mid_flush):
    """Trainer.enable_deferred_adam: each step's Adam runs at the start of the next step on a side stream,
    overlapped with that forward (per-bucket waits, the weight splits issued once their bucket is final).
    After flush() the parameters and Adam moments equal the plain trainer's bit for bit (config 4 with all
    terms, deterministic warp-loss mode); the loss of every step matches too (the forward sees the same
    parameters; up to the other loss kernels' fp64 atomics' summation order).  mid_flush: flush() after every
    other step, as a checkpoint save (checkpoint.Saver) or a parameter read-out does mid-training -- the captured
    graph's owed update must then not be applied a second time."""
    from tf_depth_estimation_amd import _api, train, variables
    steps = 3 if not mid_flush else 4

    def run(deferred):
        variables.get_store().reset(seed=1)
        _api.clear_programs()
        B, H, W = 2, 64, 96
        if cfg == "config2":
            tr = train.DepthOnlyTrainer(B, H, W)
            g = np.random.default_rng(9)
            tr.set_batch(torch.tensor(g.uniform(-0.5, 0.5, (B, H, W, 3)), dtype=torch.float32).cuda(),
                         torch.tensor(g.uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32).cuda())
        else:
            tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
            lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
            tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                         torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(),
                         small_pose(B, 4).cuda())
        tr.enable_wgrad_overlap()
        if deferred:
            tr.enable_deferred_adam(first_mb=0.25)
        losses = []
        if graph:
            tr.capture(warmup=1)
            losses.append(tr.total_loss())
        for k in range(steps):
            tr.step()
            torch.cuda.synchronize()
            losses.append(tr.total_loss())
            if mid_flush and k % 2 == 0:
                tr.flush()
        tr.flush()
        torch.cuda.synchronize()
        return losses, [(c.flat.clone(), c.adam_m.clone(), c.adam_v.clone()) for c in tr.chunks]

    l0, ref = run(False)
    l1, got = run(True)
    # loss values: fp64 sums of block partials added with atomics (last-bit order noise only)
    np.testing.assert_allclose(l1, l0, rtol=1e-12)
    for (a, b, c), (x, y, z) in zip(ref, got):
        assert torch.equal(a, x) and torch.equal(b, y) and torch.equal(c, z)


@pytest.mark.parametrize("wgrad", [False, True], ids=["wgrad_inline", "wgrad_side"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_net_overlap_matches_serial(graph, wgrad):
    """Trainer.enable_net_overlap (config 4): depth_net's forward and backward calls on a second stream beside
    disp_net's (a parallel graph branch under capture) give the serial step's parameters, gradients and Adam
    moments bit for bit after two steps -- the programs share nothing, and each program's calls keep their
    order.  All loss terms, deterministic warp-loss mode."""
    from tf_depth_estimation_amd import _api, train, variables

    def run(overlap):
        variables.get_store().reset(seed=1)
        _api.clear_programs()
        B, H, W = 2, 64, 96
        tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
        lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
        tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                     torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(),
                     small_pose(B, 4).cuda())
        if wgrad:
            tr.enable_wgrad_overlap()
        if overlap:
            tr.enable_net_overlap()
        if graph:
            tr.capture(warmup=1)
        for _ in range(2):
            tr.step()
        torch.cuda.synchronize()
        return tr.total_loss(), [(c.flat.clone(), c.grad.clone(), c.adam_m.clone(), c.adam_v.clone())
                                 for c in tr.chunks]

    l0, ref = run(False)
    l1, got = run(True)
    np.testing.assert_allclose(l1, l0, rtol=1e-12)
    for a, b in zip(ref, got):
        assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_net_overlap_rejects_exchange_hooks():
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    tr = train.DepthThenCamTrainer(2, 64, 96)
    tr.enable_adam_overlap(bucket_mb=0.5)
    with pytest.raises(ValueError):
        tr.enable_net_overlap()


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_deterministic_warp_scatter(graph):
    """Trainer.enable_deterministic (tde_warp_loss det_ws): the config-4 step with every loss term on
    (consistency weight 20, whose gather gradient scatters into the other view's disparity) is run-to-run
    bit-identical -- gradients, parameters, moments -- and agrees with the float-atomic mode to rounding."""
    from tf_depth_estimation_amd import _api, train, variables

    def run(det):
        variables.get_store().reset(seed=1)
        _api.clear_programs()
        B, H, W = 2, 64, 96
        tr = train.DepthThenCamTrainer(B, H, W)
        if det:
            tr.enable_deterministic()
        lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
        lab[np.random.default_rng(4).uniform(size=lab.shape) < 0.05] = np.nan
        tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                     torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(),
                     small_pose(B, 4).cuda())
        tr.enable_wgrad_overlap()
        if graph:
            tr.capture(warmup=1)
        tr.step()
        torch.cuda.synchronize()
        grads = [c.grad.clone() for c in tr.chunks]
        tr.step()
        torch.cuda.synchronize()
        return tr.loss_parts(), grads, [(c.flat.clone(), c.adam_m.clone(), c.adam_v.clone()) for c in tr.chunks]

    pa, ga, sa = run(True)
    pb, gb, sb = run(True)
    # loss VALUES: the other loss kernels (smoothness / depth pyramid) still add fp64 block sums with atomics
    # (last-bit order noise in the reported value only; no gradient depends on them)
    for k in pa:
        assert abs(pa[k] - pb[k]) <= 1e-12 * abs(pa[k]), k
    assert pa["consist"] == pb["consist"] and pa["photo"] == pb["photo"], "warp-loss parts must be bit-identical"
    for x, y in zip(ga, gb):
        assert torch.equal(x, y), "deterministic gradients differ between runs"
    for a, b in zip(sa, sb):
        assert all(torch.equal(x, y) for x, y in zip(a, b))
    if not graph:
        # first-step gradients only: after an Adam step (TF's first update is ~lr*sign(g)) near-zero gradients
        # that the two summations round differently have already moved the parameters apart
        _, gf, _ = run(False)
        for x, y in zip(ga, gf):
            e = ((x.double() - y.double()).norm() / y.double().norm()).item()
            assert e <= 1e-4, f"deterministic vs atomic gradient rel-L2 {e:.2e}"


def test_warp_loss_multi_and_pose_prep_multi_match_per_call():
    """tde_warp_loss_multi (the four scales of one direction in one launch) and tde_pose_prep_multi equal the
    per-call launches: pose matrices bit-exact; loss parts, g_P and the atomically scattered g_other up to the
    float-atomic order (1e-6 relative), g_disp / g_logits (plain +=, one writer per pixel) bit-exact."""
    from tf_depth_estimation_amd import losses as Ls
    B, H, W = 3, 48, 64
    g = np.random.default_rng(31)
    K = intrinsics(B, H, W).reshape(B, 4, 9).cuda()
    pose = small_pose(B, 32).cuda()
    scales = [(H >> s, W >> s) for s in range(4)]

    def dev(a):
        return torch.tensor(a, dtype=torch.float32).cuda().contiguous()

    imgs = [(texture(B, h, w, 40 + s).cuda(), texture(B, h, w, 50 + s).cuda()) for s, (h, w) in enumerate(scales)]
    disp = [dev(g.uniform(0.3, 1.0, (B, h, w, 1))) for h, w in scales]
    disp_o = [dev(g.uniform(0.3, 1.0, (B, h, w, 1))) for h, w in scales]
    logits = [dev(g.standard_normal((B, h, w, 2))) for h, w in scales]
    res = []
    for multi in (False, True):
        P = [torch.empty(B, 12, device="cuda") for _ in range(4)]
        Kinv = [torch.empty(B, 9, device="cuda") for _ in range(4)]
        T = torch.empty(B, 16, device="cuda")
        jobs = [dict(K=K[:, s].contiguous(), T=T if s == 0 else None, P=P[s], Kinv=Kinv[s], vec=pose)
                for s in range(4)]
        if multi:
            Ls.pose_prep_multi(jobs)
        else:
            for j in jobs:
                Ls.pose_prep(j["K"], T=j["T"], P=j["P"], Kinv=j["Kinv"], vec=j["vec"])
        acc = torch.zeros(3, dtype=torch.float64, device="cuda")
        gd = [torch.full_like(x, 0.5) for x in disp]       # accumulated into (+=)
        gdo = [torch.zeros_like(x) for x in disp_o]
        gl = [torch.zeros_like(x) for x in logits]
        gP = torch.zeros(4, B, 12, dtype=torch.float64, device="cuda")
        calls = [dict(img_src=imgs[s][0], img_tgt=imgs[s][1], P=P[s], Kinv=Kinv[s], disp=disp[s], logits=logits[s],
                      disp_other=disp_o[s], photo_w=10.0, exp_w=1.0, consist_w=20.0, g_disp=gd[s], g_logits=gl[s],
                      g_other=gdo[s], g_P=gP[s]) for s in range(4)]
        if multi:
            Ls.warp_loss_multi(acc, 0, calls)
        else:
            for c in calls:
                Ls.warp_loss(acc, 0, **c)
        torch.cuda.synchronize()
        res.append(dict(P=P, Kinv=Kinv, T=T, acc=acc, gd=gd, gdo=gdo, gl=gl, gP=gP))
    a, b = res
    assert torch.equal(a["T"], b["T"])
    for s in range(4):
        assert torch.equal(a["P"][s], b["P"][s]) and torch.equal(a["Kinv"][s], b["Kinv"][s])
        assert torch.equal(a["gd"][s], b["gd"][s]) and torch.equal(a["gl"][s], b["gl"][s])
        assert torch.allclose(a["gdo"][s], b["gdo"][s], rtol=1e-6, atol=1e-9)
    assert torch.allclose(a["acc"], b["acc"], rtol=1e-9, atol=1e-12)
    assert torch.allclose(a["gP"], b["gP"], rtol=1e-9, atol=1e-12)
    with pytest.raises(Exception):
        Ls.warp_loss_multi(acc, 0, [dict(calls[0], det_ws=torch.empty(4, device="cuda"))])


def test_depth_pyramid_multi_matches_per_map():
    """tde_loss_depth_pyramid_multi (config 4's four disparity maps in one launch) vs one launch per map: the
    gradients bit-exact (each pixel has one writer), the two fp64 loss sums up to the atomic order."""
    from tf_depth_estimation_amd import losses as Ls
    B, H, W = 2, 48, 64
    g = np.random.default_rng(41)
    preds = [[torch.tensor(g.uniform(0.2, 1.0, (B, H >> s, W >> s, 1)), dtype=torch.float32).cuda()
              for s in range(4)] for _ in range(4)]
    label = torch.tensor(g.uniform(1.0, 5.0, (B, H, W)), dtype=torch.float32)
    label[0, 3, 5] = float("nan")
    label = label.cuda()
    sw = [0.5 / 2 ** s for s in range(4)]
    res = []
    for multi in (False, True):
        acc = torch.zeros(8, dtype=torch.float64, device="cuda")
        grads = [[torch.full_like(p, 0.25) for p in m] for m in preds]
        maps = [dict(preds=preds[k], grads=grads[k], acc=acc, smooth_w=sw, slot_smooth=0, recip=True)
                for k in range(3)]
        maps.append(dict(preds=preds[3], grads=grads[3], acc=acc, smooth_w=sw, slot_smooth=0, recip=True, label=label,
                         l1_w=[1.5] * 4, slot_l1=1, nonfinite=True))
        if multi:
            Ls.pyramid_multi(maps)
        else:
            for m in maps:
                Ls.pyramid(**m)
        torch.cuda.synchronize()
        res.append((acc, grads))
    (a0, g0), (a1, g1) = res
    for k in range(4):
        for s in range(4):
            assert torch.equal(g0[k][s], g1[k][s])
    assert torch.allclose(a0, a1, rtol=1e-9, atol=1e-12)
    assert a0[1].item() > 0


def test_pose_grad_spread_matches_pose_grad_and_spatial_mean_bwd():
    """tde_pose_grad_spread (config 4's two directions: pose gradient + spatial-mean backward, one launch) equals
    tde_pose_grad followed by tde_spatial_mean_bwd per direction, bit for bit (accumulating and overwriting)."""
    from tf_depth_estimation_amd import _lib
    from tf_depth_estimation_amd._lib import ptr
    B, hw = 5, 12
    g = np.random.default_rng(61)
    K = intrinsics(B, 48, 64).reshape(B, 36).contiguous().cuda()
    pose = [small_pose(B, 62 + j).cuda() for j in range(2)]
    gP = [torch.tensor(g.standard_normal((4, B, 12)), dtype=torch.float64).cuda() for _ in range(2)]
    gT = [torch.tensor(g.standard_normal((B, 16)), dtype=torch.float32).cuda() for _ in range(2)]
    lib, st = _lib.load(), _lib.stream_ptr()
    for acc in (0, 1):
        res = []
        for fused in (False, True):
            gv = [torch.full((B, 6), 0.25, device="cuda") for _ in range(2)]
            dp = [torch.full((B, 3, 4, 6), -0.5, device="cuda") for _ in range(2)]
            if fused:
                jobs = (_lib.PoseGradArgs * 2)()
                for j in range(2):
                    jobs[j] = _lib.PoseGradArgs(B, 4, ptr(pose[j]), ptr(K), 36, ptr(gP[j]), ptr(gT[j]), ptr(gv[j]), acc,
                                                ptr(dp[j]), hw, 6, acc)
                _lib.check(lib.tde_pose_grad_spread(jobs, 2, st))
            else:
                for j in range(2):
                    _lib.check(lib.tde_pose_grad(B, 4, ptr(pose[j]), ptr(K), 36, ptr(gP[j]), ptr(gT[j]), ptr(gv[j]),
                                                 acc, st))
                    _lib.check(lib.tde_spatial_mean_bwd(B, hw, 6, ptr(dp[j]), 6, acc, ptr(gv[j]), st))
            torch.cuda.synchronize()
            res.append((gv, dp))
        for j in range(2):
            assert torch.equal(res[0][0][j], res[1][0][j]) and torch.equal(res[0][1][j], res[1][1][j])
