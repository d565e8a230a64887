"""Loss-head launch helpers (fused forward + gradient kernels of libtde.so).

Every helper ADDS weight * term into a device fp64 accumulator and ADDS the term's gradient into the
given gradient tensors, so a trainer zeroes its accumulators once per step and calls these in any
order.  Reference loss code: train_depth_then_cam_lr.py:59-91,211-355, train_depth_only.py:162-219,
train_optflow_combine.py:138-240, refine_depth.py:185-215.
"""
import ctypes

import torch

from . import _lib
from ._lib import WarpLossArgs, ptr

W_CONFIG2 = dict(smooth=1.0, depth=1.0)                                   # train_depth_only.py:33-37
W_CONFIG3 = dict(smooth=0.5, data=0.5, optflow=1.0, depth=50.0)           # train_optflow_combine.py:33-37
W_CONFIG4 = dict(smooth=1.0, data=10.0, depth=20.0, exp=1.0, cam=5.0)     # train_depth_then_cam_lr.py:44-51
W_CONFIG5 = dict(smooth=2.0, data=0.2)                                    # refine_depth.py:34-36


def dptr(t, idx=0):
    """Pointer to element `idx` of an fp64 accumulator tensor."""
    return ctypes.c_void_p(t.data_ptr() + 8 * idx)


def vptr(t, coff=0):
    """Pointer to channel `coff` of the first pixel of an NHWC tensor (channel views)."""
    return ctypes.c_void_p(t.data_ptr() + 4 * coff)


def zero(*ts):
    lib, st = _lib.load(), _lib.stream_ptr()
    for t in ts:
        _lib.check(lib.tde_zero_bytes(t.numel() * t.element_size(), ptr(t), st), "zero")


class Arena:
    """Per-step scratch tensors (loss accumulators, output gradients, pose gradients) carved out of ONE
    device buffer, so a trainer clears them all with one launch (zero()) instead of one per tensor."""

    def __init__(self):
        self._specs = []
        self.buf = None

    def new(self, shape, dtype=torch.float32):
        """Reserve a tensor; returns a callable-free placeholder index resolved by finalize()."""
        self._specs.append((tuple(shape), dtype))
        return len(self._specs) - 1

    def finalize(self):
        offs, off = [], 0
        for shape, dtype in self._specs:
            n = 1
            for d in shape:
                n *= d
            nbytes = n * torch.empty((), dtype=dtype).element_size()
            offs.append((off, n))
            off += (nbytes + 255) // 256 * 256
        self.buf = torch.zeros(max(off, 256), dtype=torch.uint8, device="cuda")
        out = []
        for (shape, dtype), (o, n) in zip(self._specs, offs):
            esz = torch.empty((), dtype=dtype).element_size()
            out.append(self.buf[o:o + n * esz].view(dtype).view(shape))
        return out

    def zero(self):
        lib, st = _lib.load(), _lib.stream_ptr()
        _lib.check(lib.tde_zero_bytes(self.buf.numel(), ptr(self.buf), st), "zero arena")


def pyramid(preds, grads, acc, smooth_w, slot_smooth, recip=False, coff=0, label=None, l1_w=None, slot_l1=None,
            nonfinite=False, accumulate=True):
    """All scales of compute_smooth_loss (of channel `coff` of each preds[s], or of 1/pred) and, with a
    label, mean|nf(resize_area(label, s) - pred_s)| in ONE launch (tde_loss_depth_pyramid): the same
    fp32 expressions as smooth() + area() + l1() per scale.  preds[s] / grads[s]: NHWC [N,H>>s,W>>s,C]
    dense tensors (same C); label: full-resolution [N,H,W] / [N,H,W,1]; smooth_w / l1_w: per-scale weights."""
    a = _pyramid_args(preds, grads, acc, smooth_w, slot_smooth, recip, coff, label, l1_w, slot_l1, nonfinite,
                      accumulate)
    _lib.call("tde_loss_depth_pyramid", ctypes.byref(a), _lib.stream_ptr())


def pyramid_multi(maps):
    """Several pyramid() calls (keyword dicts of its arguments) in ONE launch (tde_loss_depth_pyramid_multi); their
    grads must be disjoint views."""
    n = len(maps)
    if not 0 < n <= _lib.PYR_MULTI_MAX:
        raise ValueError(f"1..{_lib.PYR_MULTI_MAX} maps per launch")
    arr = (_lib.DepthLoss * n)()
    for i, kw in enumerate(maps):
        arr[i] = _pyramid_args(**kw)
    _lib.call("tde_loss_depth_pyramid_multi", arr, n, _lib.stream_ptr())


def _pyramid_args(preds, grads, acc, smooth_w, slot_smooth, recip=False, coff=0, label=None, l1_w=None, slot_l1=None,
                  nonfinite=False, accumulate=True):
    n = len(preds)
    N, H, W, C = preds[0].shape
    a = _lib.DepthLoss()
    a.N, a.H, a.W, a.nscales = N, H, W, n
    for s in range(n):
        a.pred[s] = ptr(preds[s]).value + 4 * coff
        a.pred_cs[s], a.pred_co[s] = C, 0
        a.grad[s] = ptr(grads[s]).value + 4 * coff
        a.g_cs[s], a.g_co[s] = grads[s].shape[-1], 0
        a.smooth_w[s] = float(smooth_w[s])
        a.l1_w[s] = float(l1_w[s]) if l1_w is not None else 0.0
    a.recip, a.nonfinite, a.grad_accumulate = int(recip), int(nonfinite), int(accumulate)
    a.label = ptr(label) if label is not None else None
    a.loss_smooth = dptr(acc, slot_smooth)
    a.loss_l1 = dptr(acc, slot_l1) if slot_l1 is not None else None
    return a


def smooth(pred, g, weight, acc, slot, recip=False, coff=0):
    """compute_smooth_loss of channel `coff` of pred (or of 1/pred) (train_depth_then_cam_lr.py:59-68)."""
    N, H, W, C = pred.shape
    _lib.call("tde_loss_smooth2", N, H, W, ptr(pred), C, coff, int(recip), float(weight), dptr(acc, slot), ptr(g), C,
              coff, _lib.stream_ptr())


def l1(pred, label, g, weight, acc, slot, nonfinite=False, coff=0):
    """mean|nf(label - pred[..., coff])| * weight; label dense [N,H,W] or [N,H,W,1]."""
    N, H, W, C = pred.shape
    _lib.call("tde_loss_l1", N, H, W, ptr(pred), C, coff, ptr(label), int(nonfinite), float(weight),
              dptr(acc, slot), ptr(g), C, coff, _lib.stream_ptr())


def sig_l2(pred, label, g, weight, acc, slot, deltas=(2,), weights=(1.0,), sig_epsilon=1e-3, epsilon=1e-6, coff=0):
    """DeMoN scale-invariant-gradient loss of channel `coff` of pred against label (my_losses.py:78-82):
    pointwise_l2_loss(scale_invariant_gradient(pred), scale_invariant_gradient(label)) * weight."""
    N, H, W, C = pred.shape
    n = len(deltas)
    if n != len(weights) or not 1 <= n <= 8:
        raise ValueError("deltas and weights: equal lengths, 1..8 entries")
    d = (ctypes.c_int * n)(*[int(v) for v in deltas])
    w = (ctypes.c_float * n)(*[float(v) for v in weights])
    _lib.call("tde_loss_sig_l2", N, H, W, ptr(pred), C, coff, ptr(label), n, ctypes.cast(d, ctypes.c_void_p),
              ctypes.cast(w, ctypes.c_void_p), float(sig_epsilon), float(epsilon), float(weight), dptr(acc, slot),
              ptr(g), C, coff, _lib.stream_ptr())


def area(src, dst):
    N, H, W, C = src.shape
    _lib.call("tde_resize_area_fwd", N, H, W, C, ptr(src), dst.shape[1], dst.shape[2], ptr(dst), _lib.stream_ptr())


def warp_loss(acc, slot0, img_src, img_tgt, P=None, Kinv=None, disp=None, flow=None, wmask=None, logits=None,
              disp_other=None, photo_w=0.0, exp_w=0.0, consist_w=0.0, g_disp=None, g_flow=None, g_logits=None,
              g_other=None, g_P=None, det_ws=None):
    """One direction of the fused projective-warp loss head (include/tde.h tde_warp_loss).  All NHWC
    tensors are dense; acc[slot0 .. slot0+2] += (photo, exp, consist).  det_ws: a device buffer of at least
    tde_warp_loss_det_workspace_size bytes selects the deterministic (run-to-run bit-identical) scatter."""
    a = _warp_args(img_src, img_tgt, P, Kinv, disp, flow, wmask, logits, disp_other, photo_w, exp_w, consist_w,
                   g_disp, g_flow, g_logits, g_other, g_P, det_ws)
    a.loss = dptr(acc, slot0)
    _lib.call("tde_warp_loss", ctypes.byref(a), _lib.stream_ptr())


def warp_loss_multi(acc, slot0, calls):
    """Several warp_loss calls (keyword dicts of warp_loss's arguments after slot0) in ONE launch
    (tde_warp_loss_multi).  The calls must write disjoint g_disp / g_logits views, e.g. the four scales of one
    direction; each call's deterministic scatter needs its own launch, so det_ws must be absent."""
    n = len(calls)
    if not 0 < n <= _lib.WARP_MULTI_MAX:
        raise ValueError(f"1..{_lib.WARP_MULTI_MAX} calls per launch")
    arr = (WarpLossArgs * n)()
    for i, kw in enumerate(calls):
        if kw.get("det_ws") is not None:
            raise ValueError("the deterministic scatter runs per call: use warp_loss")
        arr[i] = _warp_args(**kw)
        arr[i].loss = dptr(acc, slot0)
    _lib.call("tde_warp_loss_multi", arr, n, _lib.stream_ptr())


def _warp_args(img_src, img_tgt, P=None, Kinv=None, disp=None, flow=None, wmask=None, logits=None, disp_other=None,
               photo_w=0.0, exp_w=0.0, consist_w=0.0, g_disp=None, g_flow=None, g_logits=None, g_other=None, g_P=None,
               det_ws=None):
    B, H, W, _ = img_tgt.shape
    a = WarpLossArgs()
    a.B, a.H, a.W = B, H, W
    if disp is not None:
        a.disp, a.disp_cs, a.disp_co = ptr(disp), disp.shape[-1], 0
    if flow is not None:
        a.flow, a.flow_cs, a.flow_co = ptr(flow), flow.shape[-1], 0
    a.P, a.Kinv = ptr(P), ptr(Kinv)
    a.img_src, a.img_tgt, a.wmask = ptr(img_src), ptr(img_tgt), ptr(wmask)
    if logits is not None:
        a.logits, a.logit_cs, a.logit_co = ptr(logits), logits.shape[-1], 0
    if disp_other is not None:
        a.disp_other, a.other_cs, a.other_co = ptr(disp_other), disp_other.shape[-1], 0
    a.photo_w, a.exp_w, a.consist_w = photo_w, exp_w, consist_w
    a.g_disp, a.g_flow, a.g_logits, a.g_other, a.g_P = ptr(g_disp), ptr(g_flow), ptr(g_logits), ptr(g_other), ptr(g_P)
    if det_ws is not None:
        a.det_ws, a.det_ws_bytes = ptr(det_ws), det_ws.numel() * det_ws.element_size()
    return a


def det_workspace(B, H, W):
    """Device buffer for the deterministic warp-loss scatter of one (B, H, W) call (reusable by every later call on
    the same stream at that size or smaller: each call consumes it entirely before it returns)."""
    n = _lib.load().tde_warp_loss_det_workspace_size(B, H, W)
    return torch.empty((n + 15) // 16 * 4, device="cuda", dtype=torch.float32)


def pose_prep(K, T=None, P=None, Kinv=None, vec=None, mat=None):
    B = K.shape[0]
    _lib.call("tde_pose_prep", B, ptr(vec), ptr(mat), ptr(K), ptr(T), ptr(P), ptr(Kinv), _lib.stream_ptr())


def pose_prep_multi(jobs):
    """Several pose_prep calls (keyword dicts: K, T, P, Kinv, vec, mat) in ONE launch (tde_pose_prep_multi)."""
    n = len(jobs)
    if not 0 < n <= _lib.WARP_MULTI_MAX:
        raise ValueError(f"1..{_lib.WARP_MULTI_MAX} jobs per launch")
    arr = (_lib.PosePrepArgs * n)()
    for i, j in enumerate(jobs):
        arr[i].B = j["K"].shape[0]
        arr[i].pose_vec, arr[i].pose_mat = ptr(j.get("vec")), ptr(j.get("mat"))
        arr[i].K, arr[i].T, arr[i].P, arr[i].Kinv = ptr(j["K"]), ptr(j.get("T")), ptr(j["P"]), ptr(j["Kinv"])
    _lib.call("tde_pose_prep_multi", arr, n, _lib.stream_ptr())


def new(shape, dtype=torch.float32):
    return torch.empty(shape, device="cuda", dtype=dtype)


class _SmoothLoss(torch.autograd.Function):
    """compute_smooth_loss as a differentiable op: one tde_loss_smooth2 pass per channel yields the value
    and the gradient together; backward scales the stored gradient by the upstream scalar."""

    @staticmethod
    def forward(ctx, pred):
        if pred.dtype != torch.float32 or not pred.is_cuda:
            raise TypeError("compute_smooth_loss takes a float32 CUDA tensor")
        pred = pred.contiguous()
        N, H, W, C = pred.shape
        acc = torch.zeros(1, device=pred.device, dtype=torch.float64)
        g = torch.zeros_like(pred)
        for c in range(C):      # mean over all channels = (1/C) sum of per-channel means
            smooth(pred, g, 1.0 / C, acc, 0, coff=c)
        ctx.save_for_backward(g)
        return acc[0].float()

    @staticmethod
    def backward(ctx, dl):
        (g,) = ctx.saved_tensors
        return g * dl


class _SigLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, label, deltas, weights, sig_epsilon, epsilon):
        if pred.dtype != torch.float32 or not pred.is_cuda or pred.shape[-1] != 1:
            raise TypeError("depth_sig_loss takes a float32 CUDA [N,H,W,1] prediction")
        pred = pred.contiguous()
        label = label.contiguous().reshape(pred.shape).float()
        acc = torch.zeros(1, device=pred.device, dtype=torch.float64)
        g = torch.zeros_like(pred)
        sig_l2(pred, label, g, 1.0, acc, 0, deltas, weights, sig_epsilon, epsilon)
        ctx.save_for_backward(g)
        return acc[0].float()

    @staticmethod
    def backward(ctx, dl):
        (g,) = ctx.saved_tensors
        return g * dl, None, None, None, None, None


def depth_sig_loss(pred, label, deltas=(2,), weights=(1.0,), sig_epsilon=1e-3, epsilon=1e-6):
    """my_losses.py:78-82: pointwise_l2_loss(scale_invariant_gradient(pred), scale_invariant_gradient(label))
    with sig_params {'deltas': [2], 'weights': [1], 'epsilon': 0.001} and epsilon 1e-6 (:53) by default;
    the label may hold NaN holes (replace_nonfinite).  Differentiable wrt pred (one fused HIP pass)."""
    return _SigLoss.apply(pred, label, tuple(deltas), tuple(weights), sig_epsilon, epsilon)


def compute_smooth_loss(pred):
    """train_depth_then_cam_lr.py:59-68 (== train_depth_only.py:45-54, my_losses.py:27-36): second-order
    differences mean|dx2| + mean|dxdy| + mean|dydx| + mean|dy2| of an NHWC map (not edge-aware)."""
    if pred.dim() != 4 or pred.shape[1] < 3 or pred.shape[2] < 3:
        raise ValueError(f"compute_smooth_loss needs [N,H>=3,W>=3,C], got {tuple(pred.shape)}")
    return _SmoothLoss.apply(pred)
