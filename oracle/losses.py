"""Oracle restatement of the per-config loss loops and TF Adam (TEST INFRASTRUCTURE ONLY).

  * `compute_smooth_loss`      train_depth_then_cam_lr.py:59-68 (== train_depth_only.py:45-54)
  * `loss_depth_only`          train_depth_only.py:162-219            (config 2)
  * `loss_optflow_combine`     train_optflow_combine.py:138-240       (config 3, pose as a 4x4 matrix)
  * `loss_depth_then_cam_lr`   train_depth_then_cam_lr.py:211-355     (config 4)
  * `loss_refine`              refine_depth.py:185-215                (config 5, scale_factor = 1)
  * `adam_tf`                  tf.train.AdamOptimizer (train_depth_then_cam_lr.py:413-417)
  * `scale_invariant_gradient`, `pointwise_l2_loss`, `depth_sig_loss`   my_losses.py:78-82 (DeMoN sig
    loss of compute_loss_single_depth, split_training*.py:117).  lmbspecialops / depthmotionnet are
    NOT vendored in the reference (Demon_Data_loader.py:9-11): restated from their published
    definitions (DeMoN, Ummenhofer et al. 2017, eq. 3; depthmotionnet/v2/losses.py), parity unpinned.
Canonical interpretations of the broken scripts: SURVEY.md Appendix C.
"""
import numpy as np
import torch

from .geometry import (consistent_depth_loss, depth_optflow, optflow_warp, pose_vec2mat,
                       projective_inverse_warp)
from .tf_ops import replace_nonfinite, resize_area, softmax_ce2

W_CONFIG2 = dict(smooth=1.0, depth=1.0)                                   # train_depth_only.py:33-37
W_CONFIG3 = dict(smooth=0.5, data=0.5, optflow=1.0, depth=50.0)           # train_optflow_combine.py:33-37
W_CONFIG4 = dict(smooth=1.0, data=10.0, depth=20.0, exp=1.0, cam=5.0)     # train_depth_then_cam_lr.py:44-51
W_CONFIG5 = dict(smooth=2.0, data=0.2)                                    # refine_depth.py:34-36


def compute_smooth_loss(pred):
    """Second-order, not edge-aware: mean|dx2|+mean|dxdy|+mean|dydx|+mean|dy2| (:59-68)."""
    def grad(p):
        return p[:, :, 1:, :] - p[:, :, :-1, :], p[:, 1:, :, :] - p[:, :-1, :, :]
    dx, dy = grad(pred)
    dx2, dxdy = grad(dx)
    dydx, dy2 = grad(dy)
    return dx2.abs().mean() + dxdy.abs().mean() + dydx.abs().mean() + dy2.abs().mean()


def scale_invariant_gradient(f, deltas, weights, epsilon):
    """f: [N,H,W,1] -> [N,H,W,2*len(deltas)]: per delta d (weight w) the x and y components
    w (f(p+d) - f(p)) / (|f(p+d)| + |f(p)| + epsilon), 0 where p+d leaves the image (lmbspecialops
    ScaleInvariantGradient per delta, concatenated along channels as depthmotionnet.v2.losses does)."""
    f = f[..., 0]
    out = []
    for d, w in zip(deltas, weights):
        gx = torch.zeros_like(f)
        gy = torch.zeros_like(f)
        if d < f.shape[2]:
            a, b = f[:, :, :-d], f[:, :, d:]
            gx = torch.cat([w * (b - a) / (b.abs() + a.abs() + epsilon), gx[:, :, f.shape[2] - d:]], dim=2)
        if d < f.shape[1]:
            a, b = f[:, :-d], f[:, d:]
            gy = torch.cat([w * (b - a) / (b.abs() + a.abs() + epsilon), gy[:, f.shape[1] - d:]], dim=1)
        out += [gx, gy]
    return torch.stack(out, dim=-1)


def pointwise_l2_loss(inp, gt, epsilon):
    """depthmotionnet.v2.losses.pointwise_l2_loss: mean_p sqrt(sum_c nf(inp - stop_gradient(gt))^2 + eps)
    (channels last here)."""
    diff = replace_nonfinite(inp - gt.detach())
    return torch.sqrt((diff ** 2).sum(dim=-1) + epsilon).mean()


def depth_sig_loss(pred, label, deltas=(2,), weights=(1.0,), sig_epsilon=1e-3, epsilon=1e-6):
    """my_losses.py:78-82 with sig_params {'deltas': [2], 'weights': [1], 'epsilon': 0.001}, epsilon 1e-6 (:53)."""
    return pointwise_l2_loss(scale_invariant_gradient(pred, deltas, weights, sig_epsilon),
                             scale_invariant_gradient(label, deltas, weights, sig_epsilon), epsilon)


def _scale_hw(H, W, s):
    return int(H / (2 ** s)), int(W / (2 ** s))


def loss_depth_only(disps, label, w=W_CONFIG2, num_scales=4):
    """Config 2 (train_depth_only.py:162-219): smoothness on the disparity itself + L1 to the
    area-downsampled label, both weighted 1/2^s.  Returns (total, parts)."""
    H, W = label.shape[1], label.shape[2]
    smooth = depth = 0.0
    for s in range(num_scales):
        smooth = smooth + w["smooth"] / 2 ** s * compute_smooth_loss(disps[s])
        lab = resize_area(label, *_scale_hw(H, W, s))
        depth = depth + (lab - disps[s]).abs().mean() * w["depth"] / 2 ** s
    return depth + smooth, dict(depth=depth, smooth=smooth)


def loss_optflow_combine(outs, img_l, img_r, label, intr_ms, tgt2src, w=W_CONFIG3, num_scales=4):
    """Config 3 (train_optflow_combine.py:138-240).  outs = nets_depth.disp_net's 8 tensors;
    tgt2src [B,4,4] (format='matrix' semantics)."""
    H, W = img_l.shape[1], img_l.shape[2]
    disp = outs[:num_scales]
    fx = [o[..., 0:1] for o in outs[num_scales:]]
    fy = [o[..., 1:2] for o in outs[num_scales:]]
    smooth = smooth_x = smooth_y = depth = pixel = optflow = 0.0
    for s in range(num_scales):
        smooth = smooth + w["smooth"] / 2 ** s * compute_smooth_loss(disp[s])
        smooth_x = smooth_x + w["smooth"] / 2 ** s * compute_smooth_loss(fx[s])
        smooth_y = smooth_y + w["smooth"] / 2 ** s * compute_smooth_loss(fy[s])
        hw = _scale_hw(H, W, s)
        lab, il, ir = resize_area(label, *hw), resize_area(img_l, *hw), resize_area(img_r, *hw)
        depth = depth + (lab - disp[s]).abs().mean() * w["depth"] / 2 ** s
        _, coords_gt, wmask, _, _ = projective_inverse_warp(ir, (1.0 / lab)[..., 0], tgt2src,
                                                            intr_ms[:, s], format="matrix")
        wmask3 = torch.cat([wmask] * 3, -1)
        proj_d, _, _, _, _ = projective_inverse_warp(ir, (1.0 / disp[s])[..., 0], tgt2src,
                                                     intr_ms[:, s], format="matrix")
        pixel = pixel + ((proj_d - il).abs() * wmask3).mean() * w["data"] / 2 ** s
        proj_f = optflow_warp(ir, fx[s], fy[s])
        pixel = pixel + ((proj_f - il).abs() * wmask3).mean() * w["data"] / 2 ** s
        gfx, gfy = depth_optflow(coords_gt)
        optflow = optflow + (fx[s] - gfx).abs().mean() * w["optflow"] / 2 ** s
        optflow = optflow + (fy[s] - gfy).abs().mean() * w["optflow"] / 2 ** s
    smooth = smooth + smooth_x + smooth_y
    total = depth + smooth + optflow + pixel
    return total, dict(depth=depth, smooth=smooth, optflow=optflow, pixel=pixel)


def loss_depth_then_cam_lr(d_single_l, d_single_r, d_pair_l, d_pair_r, pose_r, pose_l, logits_l,
                           logits_r, img_l, img_r, label, intr_ms, gt_cam, w=W_CONFIG4, num_scales=4):
    """Config 4 (train_depth_then_cam_lr.py:211-355).  pose_* are depth_net's [B,1,6] outputs,
    gt_cam = concat(translation, rotation) [B,6] (:118)."""
    H, W = img_l.shape[1], img_l.shape[2]
    smooth = depth = pixel = exp = cam = consist = 0.0
    for s in range(num_scales):
        for d in (d_pair_l, d_pair_r, d_single_l, d_single_r):
            smooth = smooth + w["smooth"] / 2 ** s * compute_smooth_loss(1.0 / d[s])
        hw = _scale_hw(H, W, s)
        lab, il, ir = resize_area(label, *hw), resize_area(img_l, *hw), resize_area(img_r, *hw)
        depth = depth + replace_nonfinite(lab - d_single_l[s]).abs().mean() * w["depth"]
        proj_l, coords_r, _, z_r, T_lr = projective_inverse_warp(ir, (1.0 / d_pair_l[s])[..., 0],
                                                                 pose_r[:, 0, :], intr_ms[:, s])
        err_l = (proj_l - il).abs()
        proj_r, coords_l, _, z_l, T_rl = projective_inverse_warp(il, (1.0 / d_pair_r[s])[..., 0],
                                                                 pose_l[:, 0, :], intr_ms[:, s])
        err_r = (proj_r - ir).abs()
        if s == 0:
            T_gt = pose_vec2mat(gt_cam, "angleaxis")
            cam = cam + ((T_gt - T_lr) ** 2).mean() * w["cam"]
            cam = cam + ((torch.linalg.inv(T_gt) - T_rl) ** 2).mean() * w["cam"]
        ref = torch.zeros(logits_l[s].shape[:3] + (2,), dtype=img_l.dtype)
        ref[..., 1] = 1.0                                            # get_reference_explain_mask :76-85
        lg_l = logits_l[s][..., 0:2]
        exp = exp + w["exp"] * softmax_ce2(lg_l, ref).mean()
        p_l = torch.softmax(lg_l, -1)[..., 1:2]
        pixel = pixel + (err_l * p_l).mean() * w["data"]
        lg_r = logits_r[s][..., 0:2]
        exp = exp + w["exp"] * softmax_ce2(lg_r, ref).mean()
        p_r = torch.softmax(lg_r, -1)[..., 1:2]
        pixel = pixel + (err_r * p_r).mean() * w["data"]
        r_err = consistent_depth_loss(1.0 / d_pair_r[s], z_r, coords_r)
        l_err = consistent_depth_loss(1.0 / d_pair_l[s], z_l, coords_l)
        consist = consist + (r_err * p_l).mean() * w["depth"]
        consist = consist + (l_err * p_r).mean() * w["depth"]
    total = pixel + smooth + exp + cam + consist + depth
    return total, dict(pixel=pixel, smooth=smooth, exp=exp, cam=cam, consist=consist, depth=depth)


def loss_refine(disps, x1, x2, gt_depth, pose4, intr_ms, scale_factor=1.0, w=W_CONFIG5, num_scales=4):
    """Config 5 (refine_depth.py:185-215) with a fixed 4x4 pose and scale_factor = 1."""
    H, W = x1.shape[1], x1.shape[2]
    smooth = pixel = 0.0
    for s in range(num_scales):
        smooth = smooth + w["smooth"] / 2 ** s * compute_smooth_loss(disps[s])
        hw = _scale_hw(H, W, s)
        src, tgt, gt = resize_area(x1, *hw), resize_area(x2, *hw), resize_area(gt_depth, *hw)
        proj, _, _, _, _ = projective_inverse_warp(tgt, (1.0 / disps[s])[..., 0], pose4 * scale_factor,
                                                   intr_ms[:, s], format="matrix")
        pixel = pixel + (src - proj).abs().mean()
        pixel = pixel + (gt - scale_factor * disps[s]).abs().mean() * w["data"] / 2 ** s
    return pixel + smooth, dict(pixel=pixel, smooth=smooth)


class AdamTF:
    """tf.train.AdamOptimizer(lr, beta1) with TF defaults beta2=0.999, eps=1e-8 (epsilon-hat form):
    lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
    theta -= lr_t * m / (sqrt(v) + eps)."""

    def __init__(self, lr=2e-4, beta1=0.9, beta2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.t = 0
        self.m, self.v = {}, {}

    def step(self, params, grads):
        self.t += 1
        lr_t = self.lr * np.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        for k, p in params.items():
            g = grads[k]
            if g is None:
                continue
            m = self.m.setdefault(k, torch.zeros_like(p))
            v = self.v.setdefault(k, torch.zeros_like(p))
            m.mul_(self.b1).add_(g * (1 - self.b1))
            v.mul_(self.b2).add_(g * g * (1 - self.b2))
            with torch.no_grad():
                p -= lr_t * m / (torch.sqrt(v) + self.eps)
