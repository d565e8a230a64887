"""GPU parity at the BASELINE shapes (BASELINE.json configs 2-5 at 192x256 / 480x640) against the float64
oracle, plus per-tensor gradient bars on the well-conditioned tensors a wiring bug would show up in.

The step tests elsewhere run at 64x96; these run the real resolutions (batch reduced where the fp64 CPU
oracle would take minutes: config 3 at batch 4 of 32, config 4 at batch 2 of 8 per GPU, config 5 at batch 1
of 2 per GPU) and hold:
  * loss values at 1e-5 relative (the consistency term 1e-4: its scatter-add runs float atomics);
  * network outputs at 1e-4 relative (north star);
  * the whole gradient vector (relative L2) within max(1e-3, 8 x the fp32 oracle's own error)
    (test_gpu_nets.check_grads_global: sign()-driven losses and training-mode BN are ill-conditioned);
  * PER TENSOR, relative L2 within max(1e-3, 8 x the fp32 oracle's own error, 8 x a conditioning probe) on EVERY
    parameter tensor (round 5; the heads, flow *_opt heads, exp/mask*, pose/pred and pose/cam_cnv7 by name as
    well): a wrong gradient in a small tensor barely moves the whole-vector norm, but fails here.  The probe is the move of the fp64
    gradient when the weights carry the GPU path's ~1e-6 forward noise (check_per_tensor)."""
import numpy as np
import pytest
import torch

from oracle import geometry as OG
from oracle import losses as OL
from oracle import nets as ON

from test_gpu_nets import check_grads_global, oracle_params_from, rel_err
from test_gpu_trainers import intrinsics, small_pose, texture

pytestmark = pytest.mark.gpu

FACTOR = 8          # fp16x3 conv math (the default), as GRAD_FACTOR[4] in test_gpu_nets


@pytest.fixture(autouse=True)
def fresh_store():
    from tf_depth_estimation_amd import _api, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    torch.set_num_threads(min(16, torch.get_num_threads()))
    yield
    _api.clear_programs()
    torch.cuda.empty_cache()


def l2rel(a, r):
    a = a.detach().double().cpu().reshape(-1)
    r = r.detach().double().cpu().reshape(-1)
    return ((a - r).norm() / max(r.norm().item(), 1e-30)).item()


PERTURB = 2e-6      # relative weight perturbation of the conditioning probe: the GPU path's per-value forward error


def perturbed(P, seed=77):
    """Oracle variables multiplied by (1 + PERTURB * N(0,1)), float64: a second fp64 evaluation at the GPU's
    forward precision measures how much these sign()-driven gradients move under such noise alone."""
    g = torch.Generator().manual_seed(seed)
    for k, v in P.vars.items():
        with torch.no_grad():
            v.mul_(1.0 + PERTURB * torch.randn(v.shape, generator=g, dtype=v.dtype))
    return P


def check_per_tensor(gpu, g64, g32, patterns, gpert=None):
    """Relative-L2 bar per selected tensor: within max(1e-3, 8 x the fp32 oracle's error, 8 x the move of the fp64
    gradient under the PERTURB probe).  A wiring bug (wrong gradient buffer, view, half of a batch) is O(1) off;
    the probe term covers tensors such as a 1-element head bias whose gradient is a cancelling sum of sign()
    terms.  Returns the checked names (at least one per pattern)."""
    checked = []
    for pat in patterns:
        names = [n for n in g64 if pat in n]
        assert names, f"no tensor matches {pat!r}"
        for n in names:
            e_gpu, e_cpu = l2rel(gpu[n], g64[n]), l2rel(g32[n], g64[n])
            e_p = l2rel(gpert[n], g64[n]) if gpert is not None else 0.0
            assert e_gpu <= max(1e-3, FACTOR * e_cpu, FACTOR * e_p), \
                f"{n}: gpu {e_gpu:.2e} vs cpu-fp32 {e_cpu:.2e}, perturbation probe {e_p:.2e}"
            checked.append(n)
    return checked


def check_all_tensors(gpu, grads):
    """The per-tensor bar on EVERY parameter tensor (conv / deconv weights, BN betas, heads; round 5): the worst
    ratio of error to bar is printed (config-4 benched step: 0.19 over 150 tensors, profiles/r05)."""
    g64, g32, gp = grads[torch.float64], grads[torch.float32], grads["pert"]
    worst = max((l2rel(gpu[n], g64[n]) / max(1e-3, FACTOR * l2rel(g32[n], g64[n]), FACTOR * l2rel(gp[n], g64[n])), n)
                for n in g64)
    print(f"per-tensor worst ratio {worst[0]:.3f} ({worst[1]}) over {len(g64)} tensors")
    assert len(check_per_tensor(gpu, g64, g32, [""], gp)) == len(g64)


def test_config2_forward_full_batch():
    """configs[1] at its exact shape: nets_optflow_depth.disp_net on 8 x 192x256 (training-mode BN)."""
    from tf_depth_estimation_amd import nets_optflow_depth as nod
    from tf_depth_estimation_amd import variables
    x = torch.tensor(np.random.default_rng(30).uniform(-0.5, 0.5, (8, 192, 256, 3)), dtype=torch.float32)
    with variables.variable_scope("model"):
        outs, ep = nod.disp_net(x.cuda(), is_training=True)
    P = oracle_params_from(ep["program"].chunk, "")
    for st in P.bn.values():
        st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
    with torch.no_grad():
        ref = ON.disp_net(P, x.double(), True, scope="model/depth_net")
    for i, (o, r) in enumerate(zip(outs, ref)):
        e = rel_err(o, r)
        assert e <= 1e-4, f"disp{i + 1}: rel err {e:.2e}"


def test_config4_step_full_resolution():
    """Config 4 (train_depth_then_cam_lr.py:123-154,211-355) at 192x256, batch 2, all loss terms."""
    from tf_depth_estimation_amd import train
    B, H, W = 2, 192, 256
    tr = train.DepthThenCamTrainer(B, H, W)
    il, ir = texture(B, H, W, 31), texture(B, H, W, 32)
    g = np.random.default_rng(33)
    lab = g.uniform(0.1, 2.0, (B, H, W, 1))
    lab[g.uniform(size=lab.shape) < 0.05] = np.nan
    lab = torch.tensor(lab, dtype=torch.float32)
    K = intrinsics(B, H, W)
    gt = small_pose(B, 34)
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), gt.cuda())
    chunks = {"s": tr.single.chunk, "p": tr.pair.chunk}
    Ps = {dt: (oracle_params_from(chunks["s"], "", dt), oracle_params_from(chunks["p"], "", dt))
          for dt in (torch.float64, torch.float32)}
    Ps["pert"] = (perturbed(oracle_params_from(chunks["s"], "", torch.float64)),
                  perturbed(oracle_params_from(chunks["p"], "", torch.float64), 78))
    tr.phase_compute()
    torch.cuda.synchronize()
    parts = tr.loss_parts()
    out = {k: [t.detach().cpu() for t in v] for k, v in tr._out.items()}
    pose_gpu = {d: tr.pose[d].detach().cpu() for d in ("lr", "rl")}
    grads = {}
    for key, (Pss, Ppp) in Ps.items():
        dt = torch.float64 if key == "pert" else key
        x = {k: v.to(dt) for k, v in dict(il=il, ir=ir).items()}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        total, rparts = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.to(dt),
                                                  K.to(dt), gt.to(dt))
        if key is torch.float64:
            for i in range(4):
                assert rel_err(out["sl"][i], dsl[i]) <= 1e-4, f"single disp{i + 1}"
                assert rel_err(out["sr"][i], dsr[i]) <= 1e-4, f"single (right) disp{i + 1}"
                assert rel_err(out["pl"][i], dpl[i]) <= 1e-4, f"pair disp{i + 1}"
                assert rel_err(out["pl"][5 + i], ml[i]) <= 1e-4, f"mask{i + 1}"
            assert rel_err(pose_gpu["lr"], pr.reshape(B, 6)) <= 1e-4, "pose lr"
            assert rel_err(pose_gpu["rl"], pl.reshape(B, 6)) <= 1e-4, "pose rl"

            def val(t):
                return t.item() if torch.is_tensor(t) else float(t)
            for k in ("smooth", "depth", "exp", "cam"):
                assert abs(parts[k] - val(rparts[k])) <= 1e-5 * abs(val(rparts[k])) + 1e-9, k
            assert abs(parts["photo"] - val(rparts["pixel"])) <= 1e-5 * val(rparts["pixel"]) + 1e-9
            assert abs(parts["consist"] - val(rparts["consist"])) <= 1e-4 * val(rparts["consist"]) + 1e-9
        total.backward()
        grads[key] = {k: v.grad for P in (Pss, Ppp) for k, v in P.vars.items()}
    gpu = {}
    for c in chunks.values():
        gpu.update({k: c.grad_view(k) for k in c.names()})
    check_grads_global(gpu, grads[torch.float64], grads[torch.float32], FACTOR)
    names = check_per_tensor(gpu, grads[torch.float64], grads[torch.float32],
                             ["model_singledepth/depth_net/disp", "model_pairdepth/depth_cam_net/disp",
                              "pose/pred", "pose/cam_cnv7/weights", "exp/mask"], grads["pert"])
    assert len(names) >= 26
    check_all_tensors(gpu, grads)


def test_config4_forward_benched_batch():
    """The exact code bench.py times for the headline (config 4 at its per-GPU batch 8, 192x256): the trainer's
    twin batching -- disp_net once over [left; right] (2B = 16 rows) and depth_net once over
    [concat(L,R); concat(R,L)], every BatchNorm row-grouped (groups=2: each half normalised over its own 8 rows,
    as the reference's separate calls, train_depth_then_cam_lr.py:130-136,146-154) -- against the fp64 oracle's
    FOUR separate calls: every network output (single and pair disparities, masks), both poses and every loss
    term.  Forward-only on the oracle side (the gradients of this path are held at batch 2 above)."""
    from tf_depth_estimation_amd import train
    B, H, W = 8, 192, 256
    tr = train.DepthThenCamTrainer(B, H, W)
    assert tr.twin and tr.runs["s"].groups == 2 and tr.runs["p"].groups == 2 and tr.runs["s"].N == 2 * B
    # bench.py's schedule at N = 1: depth_net's filter gradients on their side stream, the two networks on two
    # streams
    tr.enable_wgrad_overlap(only=["pair"])
    tr.enable_net_overlap()
    il, ir = texture(B, H, W, 51), texture(B, H, W, 52)
    g = np.random.default_rng(53)
    lab = g.uniform(0.1, 2.0, (B, H, W, 1))
    lab[g.uniform(size=lab.shape) < 0.05] = np.nan
    lab = torch.tensor(lab, dtype=torch.float32)
    K = intrinsics(B, H, W)
    gt = small_pose(B, 54)
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), gt.cuda())
    Pss = oracle_params_from(tr.single.chunk, "", torch.float64)
    Ppp = oracle_params_from(tr.pair.chunk, "", torch.float64)
    tr.phase_compute()
    torch.cuda.synchronize()
    parts = tr.loss_parts()
    out = {k: [t.detach().cpu() for t in v] for k, v in tr._out.items()}
    pose_gpu = {d: tr.pose[d].detach().cpu() for d in ("lr", "rl")}
    with torch.no_grad():
        x = {k: v.double() for k, v in dict(il=il, ir=ir).items()}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        _, rparts = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.double(),
                                              K.double(), gt.double())
    for i in range(4):
        assert rel_err(out["sl"][i], dsl[i]) <= 1e-4, f"single disp{i + 1}"
        assert rel_err(out["sr"][i], dsr[i]) <= 1e-4, f"single (right) disp{i + 1}"
        assert rel_err(out["pl"][i], dpl[i]) <= 1e-4, f"pair disp{i + 1}"
        assert rel_err(out["pr"][i], dpr[i]) <= 1e-4, f"pair (right) disp{i + 1}"
        assert rel_err(out["pl"][5 + i], ml[i]) <= 1e-4, f"mask{i + 1}"
        assert rel_err(out["pr"][5 + i], mr[i]) <= 1e-4, f"mask (right) {i + 1}"
    assert rel_err(pose_gpu["lr"], pr.reshape(B, 6)) <= 1e-4, "pose lr"
    assert rel_err(pose_gpu["rl"], pl.reshape(B, 6)) <= 1e-4, "pose rl"

    def val(t):
        return t.item() if torch.is_tensor(t) else float(t)
    for k in ("smooth", "depth", "exp", "cam"):
        assert abs(parts[k] - val(rparts[k])) <= 1e-5 * abs(val(rparts[k])) + 1e-9, k
    assert abs(parts["photo"] - val(rparts["pixel"])) <= 1e-5 * val(rparts["pixel"]) + 1e-9
    assert abs(parts["consist"] - val(rparts["consist"])) <= 1e-4 * val(rparts["consist"]) + 1e-9


@pytest.mark.timeout(900)
def test_config4_step_benched_batch():
    """The benched step's BACKWARD at its exact shape: config 4 at per-GPU batch 8, 192x256,
    twin-batched (disp_net once over [left; right], depth_net once over [concat(L,R); concat(R,L)], grouped BN),
    bench.py's N = 1 schedule (depth_net's filter gradients on their side stream, the two networks on two streams),
    against the fp64 oracle's four separate calls (train_depth_then_cam_lr.py:123-154,355,413-417): the whole
    gradient vector within max(1e-3, 8 x the fp32 oracle's error), and per tensor the heads (disp*, exp/mask*),
    pose/pred and pose/cam_cnv7 within max(1e-3, 8 x fp32 error, 8 x the conditioning probe)."""
    from tf_depth_estimation_amd import train
    B, H, W = 8, 192, 256
    tr = train.DepthThenCamTrainer(B, H, W)
    assert tr.twin and tr.runs["s"].groups == 2 and tr.runs["p"].groups == 2
    tr.enable_wgrad_overlap(only=["pair"])
    tr.enable_net_overlap()
    il, ir = texture(B, H, W, 61), texture(B, H, W, 62)
    g = np.random.default_rng(63)
    lab = g.uniform(0.1, 2.0, (B, H, W, 1))
    lab[g.uniform(size=lab.shape) < 0.05] = np.nan
    lab = torch.tensor(lab, dtype=torch.float32)
    K = intrinsics(B, H, W)
    gt = small_pose(B, 64)
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), gt.cuda())
    chunks = {"s": tr.single.chunk, "p": tr.pair.chunk}
    Ps = {dt: (oracle_params_from(chunks["s"], "", dt), oracle_params_from(chunks["p"], "", dt))
          for dt in (torch.float64, torch.float32)}
    Ps["pert"] = (perturbed(oracle_params_from(chunks["s"], "", torch.float64)),
                  perturbed(oracle_params_from(chunks["p"], "", torch.float64), 78))
    tr.phase_compute()
    torch.cuda.synchronize()
    parts = tr.loss_parts()
    gpu = {}
    for c in chunks.values():
        gpu.update({k: c.grad_view(k).detach().cpu().clone() for k in c.names()})
    grads = {}
    for key, (Pss, Ppp) in Ps.items():
        dt = torch.float64 if key == "pert" else key
        x = {k: v.to(dt) for k, v in dict(il=il, ir=ir).items()}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        total, rparts = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.to(dt),
                                                  K.to(dt), gt.to(dt))
        if key is torch.float64:
            def val(t):
                return t.item() if torch.is_tensor(t) else float(t)
            for k in ("smooth", "depth", "exp", "cam"):
                assert abs(parts[k] - val(rparts[k])) <= 1e-5 * abs(val(rparts[k])) + 1e-9, k
            assert abs(parts["photo"] - val(rparts["pixel"])) <= 1e-5 * val(rparts["pixel"]) + 1e-9
            assert abs(parts["consist"] - val(rparts["consist"])) <= 1e-4 * val(rparts["consist"]) + 1e-9
        total.backward()
        grads[key] = {k: v.grad for P in (Pss, Ppp) for k, v in P.vars.items()}
        del dsl, dsr, dpl, dpr, pr, pl, ml, mr, total
    check_grads_global(gpu, grads[torch.float64], grads[torch.float32], FACTOR)
    names = check_per_tensor(gpu, grads[torch.float64], grads[torch.float32],
                             ["model_singledepth/depth_net/disp", "model_pairdepth/depth_cam_net/disp",
                              "pose/pred", "pose/cam_cnv7/weights", "exp/mask"], grads["pert"])
    assert len(names) >= 26
    check_all_tensors(gpu, grads)


def test_config3_step_full_resolution():
    """Config 3 (train_optflow_combine.py:97-240) at 192x256, batch 4 of the per-GPU 32."""
    from tf_depth_estimation_amd import train
    B, H, W = 4, 192, 256
    tr = train.OptflowCombineTrainer(B, H, W)
    il, ir = texture(B, H, W, 35), texture(B, H, W, 36)
    lab = torch.tensor(np.random.default_rng(37).uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32)
    K = intrinsics(B, H, W)
    T = OG.pose_vec2mat((small_pose(B, 38) * torch.tensor([0.1, 0.1, 0.1, 1, 1, 1])).double(), "angleaxis").float()
    tr.set_batch(il.cuda(), ir.cuda(), lab.cuda(), K.cuda(), T.cuda())
    Ps = {dt: oracle_params_from(tr.prog.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    Ps["pert"] = perturbed(oracle_params_from(tr.prog.chunk, "", torch.float64))
    tr.phase_compute()
    torch.cuda.synchronize()
    gouts = [t.detach().cpu() for t in (tr.run.view_tensor(v) for v in tr.prog.spec.outputs)]
    grads = {}
    for key, P in Ps.items():
        dt = torch.float64 if key == "pert" else key
        outs = ON.disp_net_depthflow(P, torch.cat([il, ir], -1).to(dt), True, scope="model/depth_net")
        total, _ = OL.loss_optflow_combine(outs, il.to(dt), ir.to(dt), lab.to(dt), K.to(dt), T.to(dt))
        if key is torch.float64:
            for i, (o, r) in enumerate(zip(gouts, outs)):
                assert rel_err(o, r) <= 1e-4, f"output {i}"
            assert abs(tr.total_loss() - total.item()) <= 1e-5 * total.item()
        total.backward()
        grads[key] = {k: v.grad for k, v in P.vars.items()}
    gpu = {k: tr.prog.chunk.grad_view(k) for k in tr.prog.chunk.names()}
    check_grads_global(gpu, grads[torch.float64], grads[torch.float32], FACTOR)
    check_per_tensor(gpu, grads[torch.float64], grads[torch.float32],
                     ["model/depth_net/disp1/", "model/depth_net/disp2/", "model/depth_net/disp3/",
                      "model/depth_net/disp4/", "_opt/"], grads["pert"])
    check_all_tensors(gpu, grads)


def test_config5_forward_and_step_640x480():
    """Config 5 (refine_depth.py:185-215, canonical interpretation) at 480x640, batch 1."""
    from tf_depth_estimation_amd import train
    B, H, W = 1, 480, 640
    tr = train.RefineTrainer(B, H, W)
    x1, x2 = texture(B, H, W, 39), texture(B, H, W, 40)
    gt = torch.tensor(np.random.default_rng(41).uniform(0.25, 4.0, (B, H, W, 1)), dtype=torch.float32)
    K = intrinsics(B, H, W)
    T = OG.pose_vec2mat((small_pose(B, 42) * torch.tensor([0.1, 0.1, 0.1, 1, 1, 1])).double(), "angleaxis").float()
    tr.set_batch(x1.cuda(), x2.cuda(), gt.cuda(), K.cuda(), T.cuda())
    Ps = {dt: oracle_params_from(tr.prog.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    Ps["pert"] = perturbed(oracle_params_from(tr.prog.chunk, "", torch.float64))
    tr.phase_compute()
    torch.cuda.synchronize()
    gouts = [t.detach().cpu() for t in (tr.run.view_tensor(v) for v in tr.prog.spec.outputs)]
    grads = {}
    for key, P in Ps.items():
        dt = torch.float64 if key == "pert" else key
        d = ON.disp_net(P, x1.to(dt), True, scope="model/depth_net")
        total, _ = OL.loss_refine(d, x1.to(dt), x2.to(dt), gt.to(dt), T.to(dt), K.to(dt))
        if key is torch.float64:
            for i, (o, r) in enumerate(zip(gouts, d)):
                assert rel_err(o, r) <= 1e-4, f"disp{i + 1}"
            assert abs(tr.total_loss() - total.item()) <= 1e-5 * total.item()
        total.backward()
        grads[key] = {k: v.grad for k, v in P.vars.items()}
    gpu = {k: tr.prog.chunk.grad_view(k) for k in tr.prog.chunk.names()}
    check_grads_global(gpu, grads[torch.float64], grads[torch.float32], FACTOR)
    check_per_tensor(gpu, grads[torch.float64], grads[torch.float32], ["model/depth_net/disp"], grads["pert"])
    check_all_tensors(gpu, grads)
