"""Pins the CPU oracle: known-answer tests from the reference formulas, NumPy-loop
cross-checks of every TF-1 op's index arithmetic, and float64 finite-difference gradient checks."""
import math

import numpy as np
import pytest
import torch

from oracle import geometry as G
from oracle import losses as L
from oracle import np_loops as NL
from oracle import tf_ops as T


@pytest.fixture(autouse=True)
def _float64_default():
    """float64 default only inside this module's tests (never leak into other test modules)."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    yield
    torch.set_default_dtype(old)


def t(a):
    return torch.tensor(np.asarray(a), dtype=torch.float64)


# ---------------------------------------------------------------- SAME padding (Appendix B.1)
@pytest.mark.parametrize("n,k,s,exp", [(192, 7, 2, (96, 2, 3)), (96, 5, 2, (48, 1, 2)), (48, 3, 2, (24, 0, 1)),
                                       (3, 3, 2, (2, 1, 1)), (96, 7, 1, (96, 3, 3)), (480, 7, 2, (240, 2, 3))])
def test_same_pad_kat(n, k, s, exp):
    assert T.same_pad(n, k, s) == exp


@pytest.mark.parametrize("H,W,C,K,k,s", [(5, 7, 3, 4, 3, 1), (6, 8, 2, 3, 3, 2), (7, 5, 3, 2, 7, 2),
                                         (3, 4, 4, 2, 3, 2), (9, 9, 2, 2, 5, 2), (2, 2, 3, 2, 3, 1)])
def test_conv2d_same_vs_loops(H, W, C, K, k, s):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, H, W, C)); w = rng.standard_normal((k, k, C, K))
    np.testing.assert_allclose(T.conv2d_same(t(x), t(w), s).numpy(), NL.conv2d_same(x, w, s), atol=1e-12)


@pytest.mark.parametrize("h,w_,C,K,k", [(2, 2, 3, 2, 3), (3, 4, 2, 3, 3), (3, 2, 2, 2, 5), (2, 3, 2, 2, 7), (1, 1, 2, 3, 3)])
def test_conv2d_transpose_vs_loops(h, w_, C, K, k):
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, h, w_, C)); w = rng.standard_normal((k, k, K, C))
    np.testing.assert_allclose(T.conv2d_transpose_same(t(x), t(w), 2).numpy(),
                               NL.conv2d_transpose_same(x, w, 2), atol=1e-12)


def test_conv2d_transpose_is_adjoint_of_conv():
    """<conv(y), x> == <y, conv_transpose(x)> for the virtual forward conv (s*h -> h)."""
    rng = np.random.default_rng(2)
    for k in (3, 5, 7):
        y = t(rng.standard_normal((1, 8, 6, 3))); x = t(rng.standard_normal((1, 4, 3, 2)))
        w = t(rng.standard_normal((k, k, 3, 2)))
        lhs = (T.conv2d_same(y, w, 2) * x).sum()
        rhs = (y * T.conv2d_transpose_same(x, w, 2)).sum()
        assert abs(lhs - rhs) < 1e-9


# ---------------------------------------------------------------- resize ops (Appendix B.5-7)
def test_resize_bilinear_kat():
    x = t([[1.0, 3.0]]).reshape(1, 1, 2, 1)
    y = T.resize_bilinear_legacy(x, 1, 4).reshape(-1).numpy()
    np.testing.assert_allclose(y, [1.0, 2.0, 3.0, 3.0])      # [a,(a+b)/2,b,b]


def test_resize_nearest_kat():
    x = t(np.arange(4.0)).reshape(1, 4, 1, 1)
    y = T.resize_nearest_legacy(x, 3, 1).reshape(-1).numpy()
    np.testing.assert_allclose(y, [0.0, 1.0, 2.0])          # rows 0,1,2
    x = t(np.arange(16.0)).reshape(1, 16, 1, 1)
    assert T.resize_nearest_legacy(x, 15, 1).reshape(-1).numpy()[-1] == 14.0


@pytest.mark.parametrize("shape,out", [((2, 3, 4, 2), (6, 8)), ((1, 4, 4, 1), (3, 4)), ((1, 16, 20, 3), (15, 20)),
                                       ((2, 5, 3, 1), (10, 6))])
def test_resize_vs_loops(shape, out):
    x = np.random.default_rng(3).standard_normal(shape)
    np.testing.assert_allclose(T.resize_bilinear_legacy(t(x), *out).numpy(), NL.resize_bilinear(x, *out), atol=1e-12)
    np.testing.assert_allclose(T.resize_nearest_legacy(t(x), *out).numpy(), NL.resize_nearest(x, *out), atol=1e-12)


def test_resize_area_kat():
    x = t(np.arange(16.0)).reshape(1, 4, 4, 1)
    np.testing.assert_allclose(T.resize_area(x, 2, 2).reshape(-1).numpy(), [2.5, 4.5, 10.5, 12.5])
    x[0, 0, 0, 0] = float("nan")
    assert math.isnan(T.resize_area(x, 2, 2)[0, 0, 0, 0].item())


# ---------------------------------------------------------------- batch norm
def test_batch_norm_train_and_moving_stats():
    rng = np.random.default_rng(4)
    x = t(rng.standard_normal((2, 3, 4, 5)) * 3 + 1)
    beta = t(rng.standard_normal(5))
    st = T.BNState(5)
    y = T.batch_norm(x, beta, st, True, 0.99)
    xn = x.numpy().reshape(-1, 5)
    m, v = xn.mean(0), xn.var(0)
    np.testing.assert_allclose(y.numpy().reshape(-1, 5), (xn - m) / np.sqrt(v + 1e-3) + beta.numpy(), atol=1e-12)
    np.testing.assert_allclose(st.moving_mean.numpy(), 0.01 * m, atol=1e-12)
    np.testing.assert_allclose(st.moving_variance.numpy(), 0.99 + 0.01 * v * 24 / 23, atol=1e-12)
    y2 = T.batch_norm(x, beta, st, False, 0.99)
    np.testing.assert_allclose(y2.numpy().reshape(-1, 5),
                               (xn - st.moving_mean.numpy()) / np.sqrt(st.moving_variance.numpy() + 1e-3) + beta.numpy())


# ---------------------------------------------------------------- geometry KATs (§8c)
def test_pose_vec2mat_rz():
    th = 0.3
    T4 = G.pose_vec2mat(t([[1.0, 2.0, 3.0, 0.0, 0.0, th]]), "angleaxis")[0].numpy()
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    np.testing.assert_allclose(T4[:3, :3], Rz, atol=1e-12)
    np.testing.assert_allclose(T4[:3, 3], [1, 2, 3])
    np.testing.assert_allclose(T4[3], [0, 0, 0, 1])


def test_pose_vec2mat_rodrigues_orthonormal():
    r = np.random.default_rng(5).standard_normal((4, 6)) * 0.3
    R = G.pose_vec2mat(t(r))[:, :3, :3].numpy()
    for Ri in R:
        np.testing.assert_allclose(Ri @ Ri.T, np.eye(3), atol=1e-12)
        assert abs(np.linalg.det(Ri) - 1) < 1e-12


def test_pose_vec2mat_zero_rotation_is_nan():
    """The reference divides by ||r|| without a guard (utils_lr.py:129-132)."""
    T4 = G.pose_vec2mat(t([[0.1, 0, 0, 0, 0, 0]]))
    assert torch.isnan(T4[0, :3, :3]).all()


def test_meshgrid_integer_pixels():
    g = G.meshgrid(1, 3, 5)[0].numpy()
    np.testing.assert_allclose(g[0, 1], [0, 1, 2, 3, 4], atol=1e-12)
    np.testing.assert_allclose(g[1, :, 2], [0, 1, 2], atol=1e-12)


def _K(B, H, W):
    fx, fy = 0.89 * W, 1.19 * H
    return G.make_intrinsics_matrix(t([fx] * B), t([fy] * B), t([0.5 * W] * B), t([0.5 * H] * B))


def test_identity_warp_returns_image():
    rng = np.random.default_rng(6)
    B, H, W = 2, 6, 8
    img = t(rng.standard_normal((B, H, W, 3)))
    depth = t(rng.uniform(1, 3, (B, H, W)))
    out, coords, wmask, z, _ = G.projective_inverse_warp(img, depth, torch.eye(4).expand(B, 4, 4), _K(B, H, W), "matrix")
    np.testing.assert_allclose(out[:, :-1, :-1].numpy(), img[:, :-1, :-1].numpy(), atol=1e-9)
    np.testing.assert_allclose(wmask[:, :-1, :-1].numpy(), 1.0, atol=1e-9)
    np.testing.assert_allclose(z[..., 0].numpy(), depth.numpy(), atol=1e-12)


def test_pure_x_translation_shift():
    B, H, W = 1, 4, 10
    depth = torch.full((B, H, W), 2.0)
    K = _K(B, H, W)
    tx = 0.05
    pose = torch.eye(4).expand(B, 4, 4).clone(); pose[:, 0, 3] = tx
    _, coords, _, _, _ = G.projective_inverse_warp(torch.zeros(B, H, W, 3), depth, pose, K, "matrix")
    shift = coords[..., 0] - G.meshgrid(B, H, W)[:, 0]
    np.testing.assert_allclose(shift.numpy(), K[0, 0, 0].item() * tx / 2.0, atol=1e-9)


def test_bilinear_sampler_kats():
    img = t(np.arange(12.0)).reshape(1, 3, 4, 1)
    def samp(x, y):
        return G.bilinear_sampler(img, t([[[[x, y]]]]))[0].item()
    assert samp(2.0, 1.0) == img[0, 1, 2, 0].item()                 # on integers -> the pixel
    assert samp(3.0, 0.0) == img[0, 0, 3, 0].item()                 # right edge pixel (unlike util.py)
    assert samp(-5.0, 1.0) == 0.0 and samp(1.0, 7.0) == 0.0         # fully out of range
    np.testing.assert_allclose(samp(-0.3, 0.0), 0.7 * img[0, 0, 0, 0].item())
    np.testing.assert_allclose(samp(0.0, -0.3), 0.7 * img[0, 0, 0, 0].item())
    img2 = img + 1.0
    np.testing.assert_allclose(G.bilinear_sampler(img2, t([[[[-0.3, 1.0]]]]))[0].item(), 0.7 * img2[0, 1, 0, 0].item())


def test_bilinear_sampler_vs_loops():
    rng = np.random.default_rng(7)
    img = rng.standard_normal((2, 5, 6, 3))
    coords = rng.uniform(-2, 8, (2, 4, 3, 2))
    coords[0, 0, 0] = [2.0, 3.0]; coords[0, 0, 1] = [5.0, 4.0]; coords[1, 1, 1] = [-1.0, 0.5]
    o, m = G.bilinear_sampler(t(img), t(coords))
    o2, m2 = NL.bilinear_sample(img, coords)
    np.testing.assert_allclose(o.numpy(), o2, atol=1e-12)
    np.testing.assert_allclose(m.numpy(), m2, atol=1e-12)


def test_bilinear_matches_grid_sample_align_corners():
    """Independent cross-check: F.grid_sample(zeros, align_corners=True)."""
    import torch.nn.functional as F
    rng = np.random.default_rng(8)
    img = t(rng.standard_normal((2, 5, 6, 3)))
    coords = t(rng.uniform(-2, 8, (2, 4, 3, 2)))
    o, _ = G.bilinear_sampler(img, coords)
    grid = torch.stack([coords[..., 0] / 5 * 2 - 1, coords[..., 1] / 4 * 2 - 1], -1)
    ref = F.grid_sample(img.permute(0, 3, 1, 2), grid, mode="bilinear", padding_mode="zeros",
                        align_corners=True).permute(0, 2, 3, 1)
    np.testing.assert_allclose(o.numpy(), ref.numpy(), atol=1e-12)


# ---------------------------------------------------------------- losses
def test_smooth_loss_of_affine_ramp_is_zero():
    yy, xx = np.meshgrid(np.arange(6.0), np.arange(7.0), indexing="ij")
    ramp = t(0.3 * xx - 0.7 * yy + 2).reshape(1, 6, 7, 1)
    assert L.compute_smooth_loss(ramp).item() < 1e-12


def test_softmax_ce_of_zero_logits_is_ln2():
    np.testing.assert_allclose(T.softmax_ce2(t([[0.0, 0.0]]), t([[0.0, 1.0]])).item(), math.log(2))


def test_replace_nonfinite_gradient_masked():
    x = t([1.0, float("nan"), -2.0, float("inf")]).requires_grad_(True)
    y = T.replace_nonfinite(x)
    y.sum().backward()
    np.testing.assert_allclose(y.detach().numpy(), [1.0, 0.0, -2.0, 0.0])
    np.testing.assert_allclose(x.grad.numpy(), [1.0, 0.0, 1.0, 0.0])


def test_adam_tf_epsilon_hat():
    p = {"w": t([1.0, -2.0])}
    opt = L.AdamTF(lr=0.1)
    opt.step(p, {"w": t([0.5, -0.25])})
    # first step: m=0.1g, v=0.001g^2 -> lr_t*m/(sqrt(v)+eps) = lr*sqrt(.001)/.1 * .1g/(sqrt(.001)|g|+eps) ~ lr*sign(g)
    np.testing.assert_allclose(p["w"].numpy(), [0.9, -1.9], atol=1e-6)


# ---------------------------------------------------------------- gradient checks (float64 FD)
def test_gradcheck_warp_chain():
    rng = np.random.default_rng(9)
    B, H, W = 1, 4, 5
    img = t(rng.standard_normal((B, H, W, 3))).requires_grad_(True)
    depth = t(rng.uniform(1, 2, (B, H, W))).requires_grad_(True)
    pose = t([[0.05, -0.02, 0.03, 0.02, -0.03, 0.04]]).requires_grad_(True)
    K = _K(B, H, W)

    def f(img, depth, pose):
        out, coords, wm, z, _ = G.projective_inverse_warp(img, depth, pose, K, "angleaxis")
        return out.sum() + 0.3 * z.sum() + 0.1 * (coords ** 2).sum()
    assert torch.autograd.gradcheck(f, (img, depth, pose), eps=1e-7, atol=1e-5)


def test_gradcheck_smooth_and_resizes():
    rng = np.random.default_rng(10)
    x = t(rng.standard_normal((1, 6, 6, 1))).requires_grad_(True)
    assert torch.autograd.gradcheck(lambda a: L.compute_smooth_loss(T.resize_bilinear_legacy(a, 12, 12)), (x,))
    assert torch.autograd.gradcheck(lambda a: T.resize_nearest_legacy(a, 4, 6).sum(), (x,))


# ---------------------------------------------------------------- DeMoN sig loss (my_losses.py:78-82)
def test_sig_known_values_and_scale_invariance():
    from oracle import losses as OL
    f = torch.tensor([[1.0, 3.0, 2.0, 2.0]], dtype=torch.float64).reshape(1, 1, 4, 1)
    s = OL.scale_invariant_gradient(f, [1, 2], [1.0, 0.5], 0.0)
    assert s.shape == (1, 1, 4, 4)
    assert torch.allclose(s[0, 0, :, 0], torch.tensor([2 / 4, -1 / 5, 0.0, 0.0], dtype=torch.float64))
    assert torch.allclose(s[0, 0, :, 2], torch.tensor([0.5 * 1 / 3, 0.5 * -1 / 5, 0.0, 0.0], dtype=torch.float64))
    assert torch.all(s[..., 1] == 0) and torch.all(s[..., 3] == 0)       # H = 1: no y neighbours
    g = torch.rand(2, 7, 9, 1, dtype=torch.float64) + 0.1
    a = OL.scale_invariant_gradient(g, [1, 2, 4], [1.0, 1.0, 1.0], 0.0)
    b = OL.scale_invariant_gradient(g * 37.5, [1, 2, 4], [1.0, 1.0, 1.0], 0.0)
    assert torch.allclose(a, b, rtol=1e-12, atol=1e-14)                  # scale invariance (eps = 0)
    assert torch.all(OL.scale_invariant_gradient(torch.full((1, 5, 5, 1), 2.0, dtype=torch.float64),
                                                 [2], [1.0], 1e-3) == 0)


def test_sig_loss_nan_holes_and_gradient():
    from oracle import losses as OL
    rng = np.random.default_rng(0)
    pred = torch.tensor(rng.uniform(0.2, 2.0, (2, 6, 7, 1)), dtype=torch.float64, requires_grad=True)
    lab = torch.tensor(rng.uniform(0.2, 2.0, (2, 6, 7, 1)), dtype=torch.float64)
    lab[0, 2, 3, 0] = float("nan")
    v = OL.depth_sig_loss(pred, lab, deltas=(1, 2), weights=(1.0, 0.5))
    assert torch.isfinite(v)
    # every pixel whose diffs all involve the hole contributes sqrt(eps) at least; loss >= sqrt(eps)
    assert v.item() >= 1e-3
    assert torch.autograd.gradcheck(lambda p: OL.depth_sig_loss(p, lab, deltas=(1, 2), weights=(1.0, 0.5)), (pred,))
