"""Network- and step-level GPU parity against the float64 oracle.

North-star tolerance (BASELINE.json): depth/flow outputs within 1e-4 relative on identical inputs
(max|gpu-ref| <= 1e-4 * max|ref| per output tensor).

Gradients: the reference computes in fp32 (TF), and these losses are ill-conditioned in fp32 -- the
L1 / second-difference terms take sign() of near-zero values and BatchNorm over the few pixels of the
deep layers amplifies rounding -- so the oracle's OWN fp32 restatement deviates from its fp64 one by
up to ~1e-1 on some tensors (measured: 5-9% max-abs even for a plain linear functional of the net
outputs, from the training-mode BN backward's cancellation).  Two fp32 evaluations with different
(equally valid) summation orders land anywhere inside that noise band -- a split-K change alone moved
one tensor from 2% to 21% -- so the step-level criterion is on the whole gradient vector:
    |g_gpu - g64| / |g64| <= max(GRAD_TOL, 4 * |g_cpu32 - g64| / |g64|)   (relative L2)
and the per-tensor form (check_grads) is kept for the better-conditioned autograd test.  Kernel-level
correctness of every backward op is pinned separately at 1e-5 (tests/test_gpu_kernels.py)."""
import numpy as np
import pytest
import torch

from oracle import losses as OL
from oracle import nets as ON
from oracle import tf_ops as T

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4
GRAD_TOL = 1e-3
# bf16x3 split-precision conv math (opt-in, tde_set_conv_math(1)) keeps ~2^-16 relative per product,
# which compounds to a few 1e-4 over 20+ conv layers: it does NOT meet the 1e-4 north-star bar and is
# held to 1e-3 on outputs and 16x (not 4x) the cpu-fp32 gradient noise.  fp32 (default) meets 1e-4.
OUT_TOL_BF16X3 = 1e-3
# bf16x6 (modes 2/3, the default: exact three-way bf16 split, six MFMAs per product, < 2^-21 per product)
# is held to the fp32 bars on every output (1e-4; measured ~1e-5) and kernel (1e-5).  Its per-conv error
# is below fp32 MFMA's in rms (2.9e-7 vs 3.5e-7 of rms(ref)) but carries a sub-ulp negative bias
# (-4e-8 of rms) from the bf16 MFMA accumulation (tests/diag_conv_err.py).  The sign()-driven step
# gradients amplify such differences chaotically: over 3 seeds of the config-4 step the whole-gradient
# error was 0.2-4.7x the oracle's own fp32 error (fp32 MFMA: 0.2-1.6x; tests/diag_grad_noise.py), so the
# step-gradient factor for these modes is 8 (for scale: cuDNN's fp32 Winograd/FFT algorithms, which the
# TF-GPU reference may select, err by ~1e-5 per conv, 30x more than either mode here).
# fp16x3 (mode 4, the library default: power-of-two-scaled two-way fp16 split, three fp16 MFMAs per product,
# <= ~3 * 2^-22 per product) is in the same accuracy class as bf16x6 and held to the same bars.
GRAD_FACTOR = {0: 4, 1: 16, 2: 8, 3: 8, 4: 8}


def rel_err(gpu, ref):
    g = gpu.detach().double().cpu()
    r = ref.detach().double().cpu()
    assert g.shape == r.shape, (g.shape, r.shape)
    return (g - r).abs().max().item() / max(r.abs().max().item(), 1e-12)


def oracle_params_from(chunk, prefix, dtype=torch.float64):
    """Oracle variable store holding exactly the product's (fp32) initial values."""
    P = ON.Params(dtype=dtype)
    for name in chunk.names():
        P.vars[name] = chunk.view(name).detach().to(dtype).cpu().clone().requires_grad_(True)
    for bn_name in chunk.bn_offsets:
        m, v = chunk.moving(bn_name)
        st = T.BNState(m.numel(), dtype=dtype)
        st.moving_mean = m.detach().to(dtype).cpu().clone()
        st.moving_variance = v.detach().to(dtype).cpu().clone()
        P.bn[bn_name] = st
    return P


def check_grads(gpu, ref64, ref32, factor=4):
    for name, r in ref64.items():
        e_gpu = rel_err(gpu[name], r)
        e_cpu32 = rel_err(ref32[name], r)
        assert e_gpu <= max(GRAD_TOL, factor * e_cpu32), f"{name}: gpu {e_gpu:.2e} vs cpu-fp32 {e_cpu32:.2e}"


def check_grads_global(gpu, ref64, ref32, factor=4):
    """Whole-gradient criterion: relative L2 error of the concatenated gradient vector,
    |g_gpu - g64| / |g64| <= max(GRAD_TOL, factor * |g_cpu32 - g64| / |g64|)."""
    names = sorted(ref64)
    g = torch.cat([gpu[n].detach().double().cpu().reshape(-1) for n in names])
    r = torch.cat([ref64[n].detach().double().cpu().reshape(-1) for n in names])
    c = torch.cat([ref32[n].detach().double().cpu().reshape(-1) for n in names])
    e_gpu = ((g - r).norm() / r.norm()).item()
    e_cpu = ((c - r).norm() / r.norm()).item()
    assert e_gpu <= max(GRAD_TOL, factor * e_cpu), f"global grad: gpu {e_gpu:.2e} vs cpu-fp32 {e_cpu:.2e}"
    return e_gpu, e_cpu


def images(N, H, W, C, seed):
    g = np.random.default_rng(seed)
    return torch.tensor(g.uniform(-0.5, 0.5, size=(N, H, W, C)), dtype=torch.float32)


@pytest.fixture(autouse=True)
def fresh_store():
    from tf_depth_estimation_amd import _api, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    yield


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["fp32", "bf16x3", "bf16x6", "bf16x6r", "fp16x3"])
def conv_math(request):
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    prev = lib.tde_get_conv_math()
    _lib.check(lib.tde_set_conv_math(request.param))
    yield request.param
    _lib.check(lib.tde_set_conv_math(prev))


@pytest.mark.parametrize("N,H,W", [(2, 64, 96), (1, 192, 256)])
def test_disp_net_forward_parity(N, H, W, conv_math):
    from tf_depth_estimation_amd import nets_optflow_depth as nod
    from tf_depth_estimation_amd import variables
    x = images(N, H, W, 3, 0)
    with variables.variable_scope("model"):
        outs, ep = nod.disp_net(x.cuda(), is_training=True)
    chunk = ep["program"].chunk
    P = oracle_params_from(chunk, "model/depth_net")
    # the product already updated its moving stats once; the oracle starts from the initial ones
    for st in P.bn.values():
        st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
    ref = ON.disp_net(P, x.double(), True, scope="model/depth_net")
    tol = OUT_TOL_BF16X3 if conv_math == 1 else OUT_TOL
    for i, (o, r) in enumerate(zip(outs, ref)):
        e = rel_err(o, r)
        assert e <= tol, f"disp{i + 1}: rel err {e:.2e}"
    # moving statistics after one training-mode call
    for bn_name, st in P.bn.items():
        m, v = chunk.moving(bn_name)
        assert rel_err(m, st.moving_mean) <= tol, bn_name
        assert rel_err(v, st.moving_variance) <= tol, bn_name


def test_depth_net_pairtest_forward_parity():
    from tf_depth_estimation_amd import nets_optflow_depth_pairtest as npt
    from tf_depth_estimation_amd import variables
    x = images(2, 64, 96, 6, 1)
    with variables.variable_scope("model_pairdepth"):
        disps, pose, masks, ep = npt.depth_net(x.cuda(), is_training=True)
    P = oracle_params_from(ep["program"].chunk, "")
    for st in P.bn.values():
        st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
    rd, rp, rm = ON.depth_net(P, x.double(), True, scope="model_pairdepth/depth_cam_net", levels=4)
    for o, r in zip(disps, rd):
        assert rel_err(o, r) <= OUT_TOL
    assert rel_err(pose, rp) <= OUT_TOL
    for o, r in zip(masks, rm):
        assert rel_err(o, r) <= OUT_TOL


def test_nets_depth_config1_forward_parity():
    """BASELINE config 1: nets_depth.disp_net on one 128x96 pair (6 channels), 8 outputs."""
    from tf_depth_estimation_amd import nets_depth, variables
    x = images(1, 96, 128, 6, 2)
    with variables.variable_scope("model"):
        outs, ep = nets_depth.disp_net(x.cuda(), is_training=True)
    assert len(outs) == 8
    P = oracle_params_from(ep["program"].chunk, "")
    for st in P.bn.values():
        st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
    ref = ON.disp_net_depthflow(P, x.double(), True, scope="model/depth_net")
    for i, (o, r) in enumerate(zip(outs, ref)):
        e = rel_err(o, r)
        assert e <= OUT_TOL, f"output {i}: rel err {e:.2e}"


def test_disp_net_inference_uses_moving_stats():
    from tf_depth_estimation_amd import nets_optflow_depth as nod
    from tf_depth_estimation_amd import variables
    x = images(2, 64, 96, 3, 3)
    with variables.variable_scope("model"):
        nod.disp_net(x.cuda(), is_training=True)          # creates + updates moving stats
        outs, ep = nod.disp_net(x.cuda(), is_training=False)
    P = oracle_params_from(ep["program"].chunk, "")
    ref = ON.disp_net(P, x.double(), False, scope="model/depth_net")
    for o, r in zip(outs, ref):
        assert rel_err(o, r) <= OUT_TOL


def test_autograd_api_gradients():
    """disp_net called through the autograd Function: d(sum of outputs)/d(input) and a weight grad."""
    from tf_depth_estimation_amd import nets_optflow_depth as nod
    from tf_depth_estimation_amd import variables
    x = images(2, 64, 96, 3, 4)
    xg = x.cuda().requires_grad_(True)
    with variables.variable_scope("model"):
        outs, ep = nod.disp_net(xg, is_training=True)
    chunk = ep["program"].chunk
    chunk.grad.zero_()
    loss = sum((o * (i + 1)).sum() for i, o in enumerate(outs))
    loss.backward()
    grads = {}
    for dt in (torch.float64, torch.float32):
        P = oracle_params_from(chunk, "", dt)
        for st in P.bn.values():
            st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
        xr = x.to(dt).requires_grad_(True)
        ref = ON.disp_net(P, xr, True, scope="model/depth_net")
        lr = sum((r * (i + 1)).sum() for i, r in enumerate(ref))
        lr.backward()
        grads[dt] = dict({k: v.grad for k, v in P.vars.items()}, input=xr.grad)
    gpu = dict({k: chunk.grad_view(k) for k in chunk.names()}, input=xg.grad)
    check_grads(gpu, grads[torch.float64], grads[torch.float32])


def test_nets_depth_linear_functional_gradients():
    """Gradient check of the joint depth+flow net alone (padded concats with w_cin < C, 2-channel
    linear flow heads, the flow decoder's `*_opt` layers) under L = sum_i <R_i, out_i> with fixed
    random R_i: no loss-head sign() terms, only the training-mode BN backward's cancellation, which
    still leaves the oracle's own fp32 gradient 5-9% (max-abs) off fp64 on some deep tensors -- so
    the whole-gradient criterion applies."""
    from tf_depth_estimation_amd import nets_depth, variables
    x = images(2, 64, 96, 6, 12)
    xg = x.cuda()
    with variables.variable_scope("model"):
        outs, ep = nets_depth.disp_net(xg, is_training=True)
    chunk = ep["program"].chunk
    chunk.grad.zero_()
    g = torch.Generator().manual_seed(5)
    R = [torch.randn(o.shape, generator=g, dtype=torch.float64) for o in outs]
    sum((o * r.float().cuda()).sum() for o, r in zip(outs, R)).backward()
    grads = {}
    for dt in (torch.float64, torch.float32):
        P = oracle_params_from(chunk, "", dt)
        for st in P.bn.values():
            st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
        ref = ON.disp_net_depthflow(P, x.to(dt), True, scope="model/depth_net")
        sum((o * r.to(dt)).sum() for o, r in zip(ref, R)).backward()
        grads[dt] = {k: v.grad for k, v in P.vars.items()}
    check_grads_global({k: chunk.grad_view(k) for k in chunk.names()}, grads[torch.float64], grads[torch.float32])


def test_config2_train_step_parity(conv_math):
    """One full config-2 step (train_depth_only.py): loss, parameter gradients, Adam update."""
    from tf_depth_estimation_amd import train
    N, H, W = 2, 64, 96
    tr = train.DepthOnlyTrainer(N, H, W)
    x = images(N, H, W, 3, 5)
    lab = torch.tensor(np.random.default_rng(6).uniform(0.25, 4.0, size=(N, H, W, 1)), dtype=torch.float32)
    tr.set_batch(x.cuda(), lab.cuda())
    Ps = {dt: oracle_params_from(tr.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    p0 = {k: v.detach().clone() for k, v in Ps[torch.float64].vars.items()}
    tr.step_eager()
    torch.cuda.synchronize()
    grads = {}
    for dt, P in Ps.items():
        ref = ON.disp_net(P, x.to(dt), True, scope="model/depth_net")
        lr, _ = OL.loss_depth_only(ref, lab.to(dt))
        lr.backward()
        grads[dt] = {k: v.grad for k, v in P.vars.items()}
        if dt == torch.float64:
            assert abs(tr.total_loss() - lr.item()) <= (1e-4 if conv_math == 1 else 1e-5) * abs(lr.item())
    check_grads_global({k: tr.chunk.grad_view(k) for k in p0}, grads[torch.float64], grads[torch.float32],
                       GRAD_FACTOR[conv_math])
    # Adam: TF's first step is ~lr*sign(g), sign-sensitive where g ~ 0, so the update is checked
    # against the oracle optimizer applied to the GPU's own gradient buffer.
    opt = OL.AdamTF(lr=2e-4)
    with torch.no_grad():
        params = {k: p0[k].clone() for k in p0}
        opt.step(params, {k: tr.chunk.grad_view(k).double().cpu() for k in p0})
    for name in p0:
        err = (tr.chunk.view(name).double().cpu() - params[name]).abs().max().item()
        assert err <= 1e-3 * 2e-4 + 1e-7, f"{name}: adam update err {err:.2e}"


def test_nets_sfm_disp_net_forward_parity(conv_math):
    """nets.disp_net (nets.py:76-147, refine_depth.py:16): 3-channel LINEAR disparity heads, 3-channel
    bilinear up-samplings in the concats (64+64+3, 32+32+3, 16+3), BN decay 0.999; training and inference."""
    from tf_depth_estimation_amd import nets, variables
    x = images(2, 64, 96, 3, 20)
    with variables.variable_scope("model"):
        outs, ep = nets.disp_net(x.cuda(), is_training=True)
    assert [tuple(o.shape) for o in outs] == [(2, 64, 96, 3), (2, 32, 48, 3), (2, 16, 24, 3), (2, 8, 12, 3)]
    chunk = ep["program"].chunk
    assert tuple(chunk.view("model/depth_net/disp1/weights").shape) == (3, 3, 16, 3)
    assert tuple(chunk.view("model/depth_net/icnv3/weights").shape) == (3, 3, 131, 64)
    P = oracle_params_from(chunk, "")
    for st in P.bn.values():
        st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
    ref = ON.disp_net_sfm(P, x.double(), True, scope="model/depth_net")
    tol = OUT_TOL_BF16X3 if conv_math == 1 else OUT_TOL
    for i, (o, r) in enumerate(zip(outs, ref)):
        e = rel_err(o, r)
        assert e <= tol, f"disp{i + 1}: rel err {e:.2e}"
    for bn_name, st in P.bn.items():     # decay 0.999 moving averages
        m, v = chunk.moving(bn_name)
        assert rel_err(m, st.moving_mean) <= tol, bn_name
        assert rel_err(v, st.moving_variance) <= tol, bn_name
    with variables.variable_scope("model", reuse=True):
        outs_i, _ = nets.disp_net(x.cuda(), is_training=False)
    P = oracle_params_from(chunk, "")
    ref_i = ON.disp_net_sfm(P, x.double(), False, scope="model/depth_net")
    for i, (o, r) in enumerate(zip(outs_i, ref_i)):
        assert rel_err(o, r) <= tol, f"inference disp{i + 1}"


def test_nets_sfm_disp_net_gradients():
    """Linear functional of the 3-channel-head net's outputs: whole-gradient criterion (BN backward)."""
    from tf_depth_estimation_amd import nets, variables
    x = images(2, 64, 96, 3, 21)
    xg = x.cuda().requires_grad_(True)
    with variables.variable_scope("model"):
        outs, ep = nets.disp_net(xg, is_training=True)
    chunk = ep["program"].chunk
    chunk.grad.zero_()
    g = torch.Generator().manual_seed(22)
    R = [torch.randn(o.shape, generator=g, dtype=torch.float64) for o in outs]
    sum((o * r.float().cuda()).sum() for o, r in zip(outs, R)).backward()
    grads = {}
    for dt in (torch.float64, torch.float32):
        P = oracle_params_from(chunk, "", dt)
        for st in P.bn.values():
            st.moving_mean.zero_(); st.moving_variance.fill_(1.0)
        xr = x.to(dt).requires_grad_(True)
        ref = ON.disp_net_sfm(P, xr, True, scope="model/depth_net")
        sum((o * r.to(dt)).sum() for o, r in zip(ref, R)).backward()
        grads[dt] = dict({k: v.grad for k, v in P.vars.items()}, input=xr.grad)
    gpu = dict({k: chunk.grad_view(k) for k in chunk.names()}, input=xg.grad)
    check_grads_global(gpu, grads[torch.float64], grads[torch.float32], GRAD_FACTOR[4])
    # the heads' own tensors per tensor (their dz also carries the gradient back from the next level's concat,
    # i.e. through a training-mode BN backward: held relative to the fp32 oracle's own error)
    check_grads({n: gpu[n] for n in grads[torch.float64] if "/disp" in n},
                {n: v for n, v in grads[torch.float64].items() if "/disp" in n},
                {n: v for n, v in grads[torch.float32].items() if "/disp" in n}, GRAD_FACTOR[4])


def test_pairtest_bn_free_disp_net_parity():
    """nets_optflow_depth_pairtest.disp_net (:76-147): normalizer commented out (:83-84), every layer is
    conv + bias + ReLU.  Outputs at 1e-4 and EVERY parameter gradient per tensor (no BatchNorm backward
    cancellation here, so the per-tensor bar applies)."""
    from tf_depth_estimation_amd import nets_optflow_depth_pairtest as npt
    from tf_depth_estimation_amd import variables
    x = images(2, 64, 96, 3, 23)
    xg = x.cuda().requires_grad_(True)
    with variables.variable_scope("model"):
        outs, ep = npt.disp_net(xg, is_training=True)
    chunk = ep["program"].chunk
    assert not chunk.bn_offsets, "BN-free net must own no BatchNorm variables"
    assert "model/depth_net/cnv1/biases" in chunk.offsets and "model/depth_net/upcnv1/biases" in chunk.offsets
    # non-zero biases so the bias path is exercised (slim initialises them to 0)
    gb = torch.Generator().manual_seed(24)
    with torch.no_grad():
        for n in chunk.names():
            if n.endswith("/biases"):
                chunk.view(n).copy_(0.05 * torch.randn(chunk.view(n).shape, generator=gb))
    with variables.variable_scope("model", reuse=True):
        outs, _ = npt.disp_net(xg, is_training=True)
    chunk.grad.zero_()
    g = torch.Generator().manual_seed(25)
    R = [torch.randn(o.shape, generator=g, dtype=torch.float64) for o in outs]
    sum((o * r.float().cuda()).sum() for o, r in zip(outs, R)).backward()
    grads, refs = {}, {}
    for dt in (torch.float64, torch.float32):
        P = oracle_params_from(chunk, "", dt)
        xr = x.to(dt).requires_grad_(True)
        ref = ON.disp_net(P, xr, True, scope="model/depth_net", bn=False)
        refs[dt] = ref
        sum((o * r.to(dt)).sum() for o, r in zip(ref, R)).backward()
        grads[dt] = dict({k: v.grad for k, v in P.vars.items()}, input=xr.grad)
    for i, (o, r) in enumerate(zip(outs, refs[torch.float64])):
        e = rel_err(o, r)
        assert e <= OUT_TOL, f"disp{i + 1}: rel err {e:.2e}"
    gpu = dict({k: chunk.grad_view(k) for k in chunk.names()}, input=xg.grad)
    check_grads(gpu, grads[torch.float64], grads[torch.float32])
