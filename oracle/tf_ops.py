"""TF-1.x op semantics restated on PyTorch-CPU tensors (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py).

All tensors are NHWC like the reference.  Functions are autograd-differentiable so the oracle's
gradients come from torch.autograd in float64; the NumPy loop versions in
oracle/np_loops.py pin the index arithmetic of each op independently.

Semantics:
  * SAME padding: out = ceil(in/s), pad_total = max((out-1)*s + k - in, 0), before = total//2.
  * conv2d_transpose SAME: out = s*in, o = s*i + k - before(k), cropped to [0, s*in).
  * slim.batch_norm: center=True, scale=False, eps=1e-3, biased batch variance for normalisation.
  * resize_bilinear / resize_nearest_neighbor: legacy (align_corners=False, no half-pixel).
  * resize_area with integer factor: exact box mean.
"""
import numpy as np
import torch
import torch.nn.functional as F


def same_pad(in_size, k, s):
    """TF 'SAME' output size and (before, after) padding (tensorflow/core/framework/common_shape_fns)."""
    out = -(-in_size // s)
    total = max((out - 1) * s + k - in_size, 0)
    return out, total // 2, total - total // 2


def conv2d_same(x, w, stride):
    """slim.conv2d(..., padding='SAME') without bias: x [N,H,W,Cin], w [kh,kw,Cin,Cout]
    (nets_optflow_depth.py:88-101)."""
    _, H, W, _ = x.shape
    kh, kw = w.shape[0], w.shape[1]
    _, pt, pb = same_pad(H, kh, stride)
    _, pl, pr = same_pad(W, kw, stride)
    xp = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb))
    y = F.conv2d(xp, w.permute(3, 2, 0, 1).contiguous(), stride=stride)
    return y.permute(0, 2, 3, 1)


def conv2d_transpose_same(x, w, stride=2):
    """slim.conv2d_transpose(..., padding='SAME'): x [N,h,w,Cin], w [kh,kw,Cout,Cin] -> [N,s*h,s*w,Cout]
    (nets_optflow_depth.py:103,109,114,119,126,133,140).  TF computes it as Conv2DBackpropInput of
    the virtual forward conv (s*h -> h), whose SAME pad is before=(k-s+... )//2 (Appendix B.2)."""
    N, h, wd, _ = x.shape
    kh, kw = w.shape[0], w.shape[1]
    H, W = stride * h, stride * wd
    _, pt, _ = same_pad(H, kh, stride)
    _, pl, _ = same_pad(W, kw, stride)
    full = F.conv_transpose2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1).contiguous(), stride=stride)
    # full index o_full = s*i + k ; TF index o = o_full - pad_before
    fh, fw = full.shape[2], full.shape[3]
    need_h, need_w = pt + H, pl + W
    if need_h > fh or need_w > fw:
        full = F.pad(full, (0, max(0, need_w - fw), 0, max(0, need_h - fh)))
    y = full[:, :, pt:pt + H, pl:pl + W]
    return y.permute(0, 2, 3, 1)


class BNState:
    """Moving statistics of one slim.batch_norm layer (non-trainable model variables)."""

    def __init__(self, c, dtype=torch.float64):
        self.moving_mean = torch.zeros(c, dtype=dtype)
        self.moving_variance = torch.ones(c, dtype=dtype)


def batch_norm(x, beta, state, is_training, decay, eps=1e-3, bessel=True):
    """slim.batch_norm(center=True, scale=False) on NHWC x (arg_scope nets_optflow_depth.py:82-87).

    Training: normalise with the biased batch variance over (N,H,W); update the moving statistics
    as `assign_moving_average` does (v -= (v - value) * (1 - decay)).  `bessel=True` reproduces
    FusedBatchNorm, whose batch_variance output (used for the moving average) carries the
    n/(n-1) correction; bessel=False reproduces the non-fused nn.moments path."""
    if is_training:
        mean = x.mean(dim=(0, 1, 2))
        var = ((x - mean) ** 2).mean(dim=(0, 1, 2))
        if state is not None:
            n = x.shape[0] * x.shape[1] * x.shape[2]
            var_upd = var * (n / max(n - 1, 1)) if bessel else var
            with torch.no_grad():
                state.moving_mean -= (state.moving_mean - mean.detach().to(state.moving_mean.dtype)) * (1 - decay)
                state.moving_variance -= (state.moving_variance - var_upd.detach().to(state.moving_variance.dtype)) * (1 - decay)
    else:
        mean = state.moving_mean.to(x.dtype)
        var = state.moving_variance.to(x.dtype)
    return (x - mean) / torch.sqrt(var + eps) + beta


def resize_nearest_legacy(x, oh, ow):
    """tf.image.resize_nearest_neighbor, align_corners=False, legacy: src = min(floor(dst*in/out), in-1)
    with the scale computed in float32 (resize_like, nets_optflow_depth.py:11-16)."""
    _, H, W, _ = x.shape
    if H == oh and W == ow:
        return x
    sy = np.float32(H) / np.float32(oh)
    sx = np.float32(W) / np.float32(ow)
    iy = [min(int(np.floor(np.float32(i) * sy)), H - 1) for i in range(oh)]
    ix = [min(int(np.floor(np.float32(j) * sx)), W - 1) for j in range(ow)]
    return x[:, iy][:, :, ix]


def resize_bilinear_legacy(x, oh, ow):
    """tf.image.resize_bilinear, align_corners=False, no half-pixel centres
    (nets_optflow_depth.py:124,131,138): src = dst*scale, y0=floor, y1=min(y0+1,in-1), lerp."""
    _, H, W, _ = x.shape
    sy = np.float32(H) / np.float32(oh)
    sx = np.float32(W) / np.float32(ow)

    def axis(n_out, n_in, s):
        src = np.array([np.float32(i) * s for i in range(n_out)], dtype=np.float32)
        i0 = np.floor(src).astype(np.int64)
        i1 = np.minimum(i0 + 1, n_in - 1)
        lerp = (src - i0.astype(np.float32)).astype(np.float64)
        return i0, i1, lerp

    y0, y1, ly = axis(oh, H, sy)
    x0, x1, lx = axis(ow, W, sx)
    ly = torch.tensor(ly, dtype=x.dtype).view(1, oh, 1, 1)
    lx = torch.tensor(lx, dtype=x.dtype).view(1, 1, ow, 1)
    top = x[:, y0][:, :, x0] * (1 - lx) + x[:, y0][:, :, x1] * lx
    bot = x[:, y1][:, :, x0] * (1 - lx) + x[:, y1][:, :, x1] * lx
    return top + (bot - top) * ly


def resize_area(x, oh, ow):
    """tf.image.resize_area with integer down-scale factors (train_depth_then_cam_lr.py:227-232):
    exact f x f box mean; NaN propagates."""
    N, H, W, C = x.shape
    fy, fx = H // oh, W // ow
    assert fy * oh == H and fx * ow == W, "integer factors only"
    if fy == 1 and fx == 1:
        return x
    return x.reshape(N, oh, fy, ow, fx, C).mean(dim=(2, 4))


def softmax_ce2(logits, labels):
    """tf.nn.softmax_cross_entropy_with_logits over the last axis (train_depth_then_cam_lr.py:87-91)."""
    return -(labels * torch.log_softmax(logits, dim=-1)).sum(-1)


def replace_nonfinite(x):
    """lmbspecialops.replace_nonfinite: x where finite else 0; gradient passes only where finite
    (train_depth_then_cam_lr.py:241)."""
    return torch.where(torch.isfinite(x), x, torch.zeros_like(x))


def glorot_uniform(rng, shape):
    """slim default weights_initializer (xavier_initializer(uniform=True)); fan_in = kh*kw*shape[-2],
    fan_out = kh*kw*shape[-1]."""
    rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    fan_in, fan_out = rf * shape[-2], rf * shape[-1]
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape)
