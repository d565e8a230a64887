"""Oracle restatement of the reference networks (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py).

Straight-line code mirroring the reference files layer by layer, written independently of the
product's layer-program builder so that a mistake in one does not hide in the other.

  * `disp_net`            nets_optflow_depth.py:76-147   (BN decay 0.99, DISP_SCALING 4, MIN_DISP 0)
  * `depth_net`           nets_optflow_depth.py:151-276  (2 scales) and
                          nets_optflow_depth_pairtest.py:151-276 (4 scales, BN default decay 0.999)
  * `disp_net_depthflow`  nets_depth.py:76-199           (BN decay 0.999, DISP_SCALING 10, MIN_DISP 0.001)
  * `disp_net_sfm`        nets.py:76-147                 (BN decay 0.999, 3-channel linear heads)
  * `disp_net(bn=False)`  nets_optflow_depth_pairtest.py:76-147 (BN-free: conv + bias + ReLU)

Parameters live in a flat dict keyed by TF variable names:
  `<scope>/<layer>/weights`, `<scope>/<layer>/biases`, `<scope>/<layer>/BatchNorm/beta`; BN moving
statistics live in a dict of `BNState` keyed by `<scope>/<layer>/BatchNorm`.
"""
import zlib

import numpy as np
import torch

from .tf_ops import (BNState, batch_norm, conv2d_same, conv2d_transpose_same, glorot_uniform,
                     resize_bilinear_legacy, resize_nearest_legacy)


class Params:
    """Variable store with TF variable_scope-like create-or-reuse semantics."""

    def __init__(self, seed=1, dtype=torch.float64):
        self.seed = seed
        self.vars = {}
        self.bn = {}
        self.dtype = dtype

    def get(self, name, shape, init):
        if name not in self.vars:
            if init == "glorot":
                # per-variable stream: independent of creation order (same rule as the product)
                rng = np.random.Generator(np.random.PCG64([self.seed, zlib.crc32(name.encode())]))
                v = glorot_uniform(rng, shape)
            else:
                v = np.zeros(shape)
            self.vars[name] = torch.tensor(v, dtype=self.dtype, requires_grad=True)
        assert tuple(self.vars[name].shape) == tuple(shape), (name, self.vars[name].shape, shape)
        return self.vars[name]

    def bn_state(self, name, c):
        if name not in self.bn:
            self.bn[name] = BNState(c, dtype=self.dtype)
        return self.bn[name]


class _Ctx:
    def __init__(self, P, scope, is_training, decay, bn):
        self.P, self.scope, self.is_training, self.decay, self.bn = P, scope, is_training, decay, bn

    def conv(self, x, cout, k, s, name, bn=None, act="relu"):
        """slim.conv2d under the net's arg_scope; heads pass normalizer_fn=None (then bias)."""
        bn = self.bn if bn is None else bn
        cin = x.shape[-1]
        w = self.P.get(f"{self.scope}/{name}/weights", (k, k, cin, cout), "glorot")
        y = conv2d_same(x, w, s)
        if bn:
            beta = self.P.get(f"{self.scope}/{name}/BatchNorm/beta", (cout,), "zeros")
            st = self.P.bn_state(f"{self.scope}/{name}/BatchNorm", cout)
            y = batch_norm(y, beta, st, self.is_training, self.decay)
        else:
            b = self.P.get(f"{self.scope}/{name}/biases", (cout,), "zeros")
            y = y + b
        if act == "relu":
            y = torch.relu(y)
        elif act == "sigmoid":
            y = torch.sigmoid(y)
        return y

    def deconv(self, x, cout, k, name):
        """slim.conv2d_transpose(stride=2) + BN + ReLU under the net's arg_scope."""
        cin = x.shape[-1]
        w = self.P.get(f"{self.scope}/{name}/weights", (k, k, cout, cin), "glorot")
        y = conv2d_transpose_same(x, w, 2)
        if self.bn:
            beta = self.P.get(f"{self.scope}/{name}/BatchNorm/beta", (cout,), "zeros")
            st = self.P.bn_state(f"{self.scope}/{name}/BatchNorm", cout)
            y = batch_norm(y, beta, st, self.is_training, self.decay)
        else:
            b = self.P.get(f"{self.scope}/{name}/biases", (cout,), "zeros")
            y = y + b
        return torch.relu(y)


def _encoder(c, x):
    cnv1 = c.conv(x, 32, 7, 2, "cnv1")
    cnv1b = c.conv(cnv1, 32, 7, 1, "cnv1b")
    cnv2 = c.conv(cnv1b, 64, 5, 2, "cnv2")
    cnv2b = c.conv(cnv2, 64, 5, 1, "cnv2b")
    cnv3 = c.conv(cnv2b, 128, 3, 2, "cnv3")
    cnv3b = c.conv(cnv3, 128, 3, 1, "cnv3b")
    cnv4 = c.conv(cnv3b, 256, 3, 2, "cnv4")
    cnv4b = c.conv(cnv4, 256, 3, 1, "cnv4b")
    cnv5 = c.conv(cnv4b, 512, 3, 2, "cnv5")
    cnv5b = c.conv(cnv5, 512, 3, 1, "cnv5b")
    cnv6 = c.conv(cnv5b, 512, 3, 2, "cnv6")
    cnv6b = c.conv(cnv6, 512, 3, 1, "cnv6b")
    return cnv1b, cnv2b, cnv3b, cnv4b, cnv5b, cnv6b


def _decoder(c, H, W, cnv1b, cnv2b, cnv3b, cnv4b, cnv5b, cnv6b, cnv7b, scale, mind, sfx="",
             head_ch=1, head_act="sigmoid", levels=4, icnv6_name=None):
    """The skip-concat decoder shared by all nets (nets_optflow_depth.py:103-144)."""
    def head(x, name):
        y = c.conv(x, head_ch, 3, 1, name, bn=False, act=head_act)
        return y * scale + mind if head_act == "sigmoid" else y

    up7 = c.deconv(cnv7b, 512, 3, "upcnv7" + sfx)
    up7 = resize_nearest_legacy(up7, cnv6b.shape[1], cnv6b.shape[2])
    icnv7 = c.conv(torch.cat([up7, cnv6b], -1), 512, 3, 1, "icnv7" + sfx)
    up6 = c.deconv(icnv7, 512, 3, "upcnv6" + sfx)
    up6 = resize_nearest_legacy(up6, cnv5b.shape[1], cnv5b.shape[2])
    icnv6 = c.conv(torch.cat([up6, cnv5b], -1), 512, 3, 1, icnv6_name or ("icnv6" + sfx))
    up5 = c.deconv(icnv6, 256, 3, "upcnv5" + sfx)
    up5 = resize_nearest_legacy(up5, cnv4b.shape[1], cnv4b.shape[2])
    icnv5 = c.conv(torch.cat([up5, cnv4b], -1), 256, 3, 1, "icnv5" + sfx)
    up4 = c.deconv(icnv5, 128, 3, "upcnv4" + sfx)
    icnv4 = c.conv(torch.cat([up4, cnv3b], -1), 128, 3, 1, "icnv4" + sfx)
    disp4 = head(icnv4, "disp4" + sfx)
    disp4_up = resize_bilinear_legacy(disp4, int(H / 4), int(W / 4))
    up3 = c.deconv(icnv4, 64, 3, "upcnv3" + sfx)
    icnv3 = c.conv(torch.cat([up3, cnv2b, disp4_up], -1), 64, 3, 1, "icnv3" + sfx)
    disp3 = head(icnv3, "disp3" + sfx)
    if levels == 2:
        return [disp3, disp4]
    disp3_up = resize_bilinear_legacy(disp3, int(H / 2), int(W / 2))
    up2 = c.deconv(icnv3, 32, 3, "upcnv2" + sfx)
    icnv2 = c.conv(torch.cat([up2, cnv1b, disp3_up], -1), 32, 3, 1, "icnv2" + sfx)
    disp2 = head(icnv2, "disp2" + sfx)
    disp2_up = resize_bilinear_legacy(disp2, H, W)
    up1 = c.deconv(icnv2, 16, 3, "upcnv1" + sfx)
    icnv1 = c.conv(torch.cat([up1, disp2_up], -1), 16, 3, 1, "icnv1" + sfx)
    disp1 = head(icnv1, "disp1" + sfx)
    return [disp1, disp2, disp3, disp4]


def disp_net(P, tgt_image, is_training=True, scope="depth_net", bn=True, decay=0.99,
             disp_scaling=4.0, min_disp=0.0, head_ch=1, head_act="sigmoid"):
    """nets_optflow_depth.disp_net (nets_optflow_depth.py:76-147).  `bn=False` gives the BN-free
    variant of nets_optflow_depth_pairtest.py:77,83-85 (slim then adds biases)."""
    H, W = tgt_image.shape[1], tgt_image.shape[2]
    c = _Ctx(P, scope, is_training, decay, bn)
    feats = _encoder(c, tgt_image)
    cnv7 = c.conv(feats[5], 512, 3, 2, "cnv7")
    cnv7b = c.conv(cnv7, 512, 3, 1, "cnv7b")
    return _decoder(c, H, W, *feats, cnv7b, disp_scaling, min_disp, head_ch=head_ch, head_act=head_act)


def disp_net_sfm(P, tgt_image, is_training=True, scope="depth_net"):
    """nets.disp_net (nets.py:76-147): the same encoder / decoder with 3-channel LINEAR disparity heads
    (activation_fn=None, normalizer_fn=None, :122-144; DISP_SCALING / MIN_DISP are not applied), 3-channel
    bilinear up-samplings in the concats, slim's default BN decay 0.999 (:77)."""
    return disp_net(P, tgt_image, is_training, scope, bn=True, decay=0.999, head_ch=3, head_act=None)


def depth_net(P, tgt_image, is_training=True, scope="depth_cam_net", levels=4, decay=None,
              disp_scaling=4.0):
    """nets_optflow_depth(_pairtest).depth_net: pair encoder, pose head (no 0.01 scale, :186), exp
    mask head, depth decoder.  levels=2 -> nets_optflow_depth.py:151-276 (decay 0.99);
    levels=4 -> nets_optflow_depth_pairtest.py:151-276 (default decay 0.999).
    Returns (disps, pose [b,1,6], masks)."""
    if decay is None:
        decay = 0.99 if levels == 2 else 0.999
    H, W = tgt_image.shape[1], tgt_image.shape[2]
    c = _Ctx(P, scope, is_training, decay, True)
    cnv1b, cnv2b, cnv3b, cnv4b, cnv5b, cnv6b = _encoder(c, tgt_image)
    cam_cnv7 = c.conv(cnv6b, 256, 3, 2, "pose/cam_cnv7")
    pose_pred = c.conv(cam_cnv7, 6, 1, 1, "pose/pred", bn=False, act=None)
    pose_final = pose_pred.mean(dim=(1, 2)).reshape(-1, 1, 6)
    eu5 = c.deconv(cnv5b, 256, 3, "exp/exp_upcnv5")
    eu4 = c.deconv(eu5, 128, 3, "exp/exp_upcnv4")
    mask4 = c.conv(eu4, 2, 3, 1, "exp/mask4", bn=False, act=None)
    eu3 = c.deconv(eu4, 64, 3, "exp/exp_upcnv3")
    mask3 = c.conv(eu3, 2, 3, 1, "exp/mask3", bn=False, act=None)
    masks = [mask3, mask4]
    if levels == 4:
        eu2 = c.deconv(eu3, 32, 5, "exp/exp_upcnv2")
        mask2 = c.conv(eu2, 2, 5, 1, "exp/mask2", bn=False, act=None)
        eu1 = c.deconv(eu2, 16, 7, "exp/exp_upcnv1")
        mask1 = c.conv(eu1, 2, 7, 1, "exp/mask1", bn=False, act=None)
        masks = [mask1, mask2, mask3, mask4]
    cnv7 = c.conv(cnv6b, 512, 3, 2, "cnv7")
    cnv7b = c.conv(cnv7, 512, 3, 1, "cnv7b")
    disps = _decoder(c, H, W, cnv1b, cnv2b, cnv3b, cnv4b, cnv5b, cnv6b, cnv7b, disp_scaling, 0.0,
                     levels=levels)
    return disps, pose_final, masks


def disp_net_depthflow(P, tgt_image, is_training=True, scope="depth_net", decay=0.999):
    """nets_depth.disp_net (nets_depth.py:76-199): shared encoder, depth decoder
    (sigmoid*10+0.001) and flow decoder (2-ch linear), 8 outputs; the flow decoder's icnv6 layer
    keeps the reference's scope name `icnv6_opt_opt` (:159)."""
    H, W = tgt_image.shape[1], tgt_image.shape[2]
    c = _Ctx(P, scope, is_training, decay, True)
    feats = _encoder(c, tgt_image)
    cnv7 = c.conv(feats[5], 512, 3, 2, "cnv7")
    cnv7b = c.conv(cnv7, 512, 3, 1, "cnv7b")
    disps = _decoder(c, H, W, *feats, cnv7b, 10.0, 0.001)
    flows = _decoder(c, H, W, *feats, cnv7b, 1.0, 0.0, sfx="_opt", head_ch=2, head_act=None,
                     icnv6_name="icnv6_opt_opt")
    return disps + flows
