"""Spec builders shared by the reference-named net modules.

Each builder lays a reference network out as a NetSpec: which layers run, which buffer/channel
slice each output is written into, and which TF variable names it owns.  The layer lists follow
nets_optflow_depth.py:88-144 (encoder + skip-concat decoder), nets_optflow_depth_pairtest.py:151-276
(depth_net with pose/exp heads) and nets_depth.py:88-191 (joint depth + flow decoders).
"""
from .program import ConvBN, Copy, Head, NetSpec, Resize, View, same_pad

ENC = [("cnv1", 32, 7, 2), ("cnv1b", 32, 7, 1), ("cnv2", 64, 5, 2), ("cnv2b", 64, 5, 1), ("cnv3", 128, 3, 2),
       ("cnv3b", 128, 3, 1), ("cnv4", 256, 3, 2), ("cnv4b", 256, 3, 1), ("cnv5", 512, 3, 2), ("cnv5b", 512, 3, 1),
       ("cnv6", 512, 3, 2), ("cnv6b", 512, 3, 1)]


def level_sizes(H, W, n=7):
    """Spatial size after each stride-2 stage (SAME: ceil)."""
    hs, ws = [H], [W]
    for _ in range(n):
        hs.append(same_pad(hs[-1], 3, 2)[0])
        ws.append(same_pad(ws[-1], 3, 2)[0])
    return hs, ws


class Decoder:
    """Concat buffers of one skip decoder (nets_optflow_depth.py:103-144).  Slot layout of each concat
    is [upconv | skip | disp_up] exactly as tf.concat orders it (fixes the weight row order)."""

    def __init__(self, spec, hs, ws, sfx, head_ch, levels):
        self.sfx = sfx
        cat = spec.concat
        self.i7, self.i7_full = cat("i7_in" + sfx, hs[6], ws[6], [512, 512])
        self.i6, self.i6_full = cat("i6_in" + sfx, hs[5], ws[5], [512, 512])
        self.i5, self.i5_full = cat("i5_in" + sfx, hs[4], ws[4], [256, 256])
        self.i4, self.i4_full = cat("i4_in" + sfx, hs[3], ws[3], [128, 128])
        self.i3, self.i3_full = cat("i3_in" + sfx, hs[2], ws[2], [64, 64, head_ch])
        if levels == 4:
            self.i2, self.i2_full = cat("i2_in" + sfx, hs[1], ws[1], [32, 32, head_ch])
            self.i1, self.i1_full = cat("i1_in" + sfx, hs[0], ws[0], [16, head_ch])

    def skip_slots(self, levels):
        """Where each encoder feature lives in this decoder: cnv1b..cnv6b (None if not consumed)."""
        return {"cnv1b": self.i2[1] if levels == 4 else None, "cnv2b": self.i3[1], "cnv3b": self.i4[1],
                "cnv4b": self.i5[1], "cnv5b": self.i6[1], "cnv6b": self.i7[1]}


def build_encoder(spec, homes, decay, bn=True, last=12):
    """cnv1..cnv6b.  `homes` maps a layer to the view it is written into (a decoder concat slot);
    other layers get a dense buffer.  Returns dict layer -> view."""
    feats = {}
    src = spec.input_view
    for name, K, k, s in ENC[:last]:
        H, W = same_pad(src.H, k, s)[0], same_pad(src.W, k, s)[0]
        dst = homes.get(name) or spec.dense(name, H, W, K)
        spec.add(ConvBN(name, src, dst, K, k, s, bn=bn, decay=decay))
        feats[name] = dst
        src = dst
    return feats


def build_decoder(spec, dec, feats, cnv7b, H, W, hs, ws, decay, head_ch, head_act, scale, offset, levels=4,
                  icnv6_name=None, bn=True):
    """upcnv7 ... disp1 (nets_optflow_depth.py:103-144).  Returns [disp1, disp2, disp3, disp4] views
    (or [disp3, disp4] for levels == 2)."""
    sfx = dec.sfx

    def up(name, src, slot, K):
        # deconv + BN + ReLU, then resize_like to the skip size when they differ (:105,110,115)
        uh, uw = 2 * src.H, 2 * src.W
        if (uh, uw) == (slot.H, slot.W):
            spec.add(ConvBN(name + sfx, src, slot, K, 3, 2, deconv=True, bn=bn, decay=decay))
        else:
            tmp = spec.dense(name + sfx + "_full", uh, uw, K)
            spec.add(ConvBN(name + sfx, src, tmp, K, 3, 2, deconv=True, bn=bn, decay=decay))
            spec.add(Resize("nearest", tmp, slot))

    def conv(name, src, K, Hh, Ww):
        dst = spec.dense(name, Hh, Ww, K)
        spec.add(ConvBN(name, src, dst, K, 3, 1, bn=bn, decay=decay))
        return dst

    def head(name, src, out_slot):
        dst = spec.dense(name + sfx, src.H, src.W, head_ch)
        spec.add(Head(name + sfx, src, dst, head_ch, 3, head_act, scale, offset))
        return dst

    up("upcnv7", cnv7b, dec.i7[0], 512)
    icnv7 = conv("icnv7" + sfx, dec.i7_full, 512, hs[6], ws[6])
    up("upcnv6", icnv7, dec.i6[0], 512)
    icnv6 = conv(icnv6_name or ("icnv6" + sfx), dec.i6_full, 512, hs[5], ws[5])
    up("upcnv5", icnv6, dec.i5[0], 256)
    icnv5 = conv("icnv5" + sfx, dec.i5_full, 256, hs[4], ws[4])
    spec.add(ConvBN("upcnv4" + sfx, icnv5, dec.i4[0], 128, 3, 2, deconv=True, bn=bn, decay=decay))
    icnv4 = conv("icnv4" + sfx, dec.i4_full, 128, hs[3], ws[3])
    disp4 = head("disp4", icnv4, None)
    spec.add(Resize("bilinear", disp4, dec.i3[2]))        # int(H/4) x int(W/4)  (:124)
    spec.add(ConvBN("upcnv3" + sfx, icnv4, dec.i3[0], 64, 3, 2, deconv=True, bn=bn, decay=decay))
    icnv3 = conv("icnv3" + sfx, dec.i3_full, 64, hs[2], ws[2])
    disp3 = head("disp3", icnv3, None)
    if levels == 2:
        return [disp3, disp4]
    spec.add(Resize("bilinear", disp3, dec.i2[2]))        # (:131)
    spec.add(ConvBN("upcnv2" + sfx, icnv3, dec.i2[0], 32, 3, 2, deconv=True, bn=bn, decay=decay))
    icnv2 = conv("icnv2" + sfx, dec.i2_full, 32, hs[1], ws[1])
    disp2 = head("disp2", icnv2, None)
    spec.add(Resize("bilinear", disp2, dec.i1[1]))        # (:138)
    spec.add(ConvBN("upcnv1" + sfx, icnv2, dec.i1[0], 16, 3, 2, deconv=True, bn=bn, decay=decay))
    icnv1 = conv("icnv1" + sfx, dec.i1_full, 16, H, W)
    disp1 = head("disp1", icnv1, None)
    return [disp1, disp2, disp3, disp4]


def check_sizes(H, W, levels=4):
    """The reference's skip concats need int(H/4) == ceil(ceil(H/2)/2) etc. (no resize_like on them)."""
    hs, ws = level_sizes(H, W)
    ok = hs[2] == int(H / 4) and ws[2] == int(W / 4)
    if levels == 4:
        ok = ok and hs[1] == int(H / 2) and ws[1] == int(W / 2)
    if not ok:
        raise ValueError(f"input {H}x{W}: decoder skip shapes mismatch (reference tf.concat would fail)")
    return hs, ws


def disp_net_spec(H, W, cin, scope="depth_net", decay=0.99, scale=4.0, offset=0.0, bn=True, head_ch=1, head_act=1):
    """nets_optflow_depth.disp_net (nets_optflow_depth.py:76-147); bn=False: the BN-free variant of
    nets_optflow_depth_pairtest.py:76-147 (conv + bias + ReLU); head_ch=3, head_act=0: nets.disp_net
    (nets.py:76-147, 3-channel linear disparity heads, BN decay 0.999)."""
    hs, ws = check_sizes(H, W)
    spec = NetSpec(scope, H, W, cin)
    dec = Decoder(spec, hs, ws, "", head_ch, 4)
    feats = build_encoder(spec, dec.skip_slots(4), decay, bn=bn)
    cnv7 = spec.dense("cnv7", hs[7], ws[7], 512)
    spec.add(ConvBN("cnv7", feats["cnv6b"], cnv7, 512, 3, 2, bn=bn, decay=decay))
    cnv7b = spec.dense("cnv7b", hs[7], ws[7], 512)
    spec.add(ConvBN("cnv7b", cnv7, cnv7b, 512, 3, 1, bn=bn, decay=decay))
    spec.outputs = build_decoder(spec, dec, feats, cnv7b, H, W, hs, ws, decay, head_ch, head_act, scale, offset, bn=bn)
    spec.end_points = feats
    return spec


def depth_net_spec(H, W, cin, levels=4, scope="depth_cam_net", decay=None, scale=4.0):
    """nets_optflow_depth_pairtest.depth_net (levels=4, :151-276) / nets_optflow_depth.depth_net
    (levels=2).  Outputs: disps (levels), pose_pred [N,h7,w7,6] (mean taken by the caller), masks."""
    if decay is None:
        decay = 0.99 if levels == 2 else 0.999
    hs, ws = check_sizes(H, W, levels)
    spec = NetSpec(scope, H, W, cin)
    dec = Decoder(spec, hs, ws, "", 1, levels)
    feats = build_encoder(spec, dec.skip_slots(levels), decay)
    # pose head (:178-186) and explainability-mask branch (:189-206): side branches off the encoder that feed only
    # the loss; tagged `branch` for the step timeline
    first_branch = len(spec.ops)
    cam = spec.dense("pose/cam_cnv7", hs[7], ws[7], 256)
    spec.add(ConvBN("pose/cam_cnv7", feats["cnv6b"], cam, 256, 3, 2, decay=decay))
    pose = spec.dense("pose/pred", hs[7], ws[7], 6)
    spec.add(Head("pose/pred", cam, pose, 6, 1, 0))
    # exp head (:189-206)
    e5 = spec.dense("exp/exp_upcnv5", 2 * hs[5], 2 * ws[5], 256)
    spec.add(ConvBN("exp/exp_upcnv5", feats["cnv5b"], e5, 256, 3, 2, deconv=True, decay=decay))
    e4 = spec.dense("exp/exp_upcnv4", 2 * e5.H, 2 * e5.W, 128)
    spec.add(ConvBN("exp/exp_upcnv4", e5, e4, 128, 3, 2, deconv=True, decay=decay))
    m4 = spec.dense("exp/mask4", e4.H, e4.W, 2)
    spec.add(Head("exp/mask4", e4, m4, 2, 3, 0))
    e3 = spec.dense("exp/exp_upcnv3", 2 * e4.H, 2 * e4.W, 64)
    spec.add(ConvBN("exp/exp_upcnv3", e4, e3, 64, 3, 2, deconv=True, decay=decay))
    m3 = spec.dense("exp/mask3", e3.H, e3.W, 2)
    spec.add(Head("exp/mask3", e3, m3, 2, 3, 0))
    masks = [m3, m4]
    if levels == 4:
        e2 = spec.dense("exp/exp_upcnv2", 2 * e3.H, 2 * e3.W, 32)
        spec.add(ConvBN("exp/exp_upcnv2", e3, e2, 32, 5, 2, deconv=True, decay=decay))
        m2 = spec.dense("exp/mask2", e2.H, e2.W, 2)
        spec.add(Head("exp/mask2", e2, m2, 2, 5, 0))
        e1 = spec.dense("exp/exp_upcnv1", 2 * e2.H, 2 * e2.W, 16)
        spec.add(ConvBN("exp/exp_upcnv1", e2, e1, 16, 7, 2, deconv=True, decay=decay))
        m1 = spec.dense("exp/mask1", e1.H, e1.W, 2)
        spec.add(Head("exp/mask1", e1, m1, 2, 7, 0))
        masks = [m1, m2, m3, m4]
    for op in spec.ops[first_branch:]:
        op.branch = 1
    cnv7 = spec.dense("cnv7", hs[7], ws[7], 512)
    spec.add(ConvBN("cnv7", feats["cnv6b"], cnv7, 512, 3, 2, decay=decay))
    cnv7b = spec.dense("cnv7b", hs[7], ws[7], 512)
    spec.add(ConvBN("cnv7b", cnv7, cnv7b, 512, 3, 1, decay=decay))
    disps = build_decoder(spec, dec, feats, cnv7b, H, W, hs, ws, decay, 1, 1, scale, 0.0, levels=levels)
    spec.outputs = disps + [pose] + masks
    spec.n_disp, spec.n_mask = len(disps), len(masks)
    spec.end_points = feats
    return spec


def depthflow_net_spec(H, W, cin, scope="depth_net", decay=0.999):
    """nets_depth.disp_net (nets_depth.py:76-199): shared encoder, depth decoder (sigmoid*10+0.001),
    flow decoder (2-ch linear, scope names '*_opt', `icnv6_opt_opt` kept verbatim :159)."""
    hs, ws = check_sizes(H, W)
    spec = NetSpec(scope, H, W, cin)
    dd = Decoder(spec, hs, ws, "", 1, 4)
    fd = Decoder(spec, hs, ws, "_opt", 2, 4)
    feats = build_encoder(spec, dd.skip_slots(4), decay)
    cnv7 = spec.dense("cnv7", hs[7], ws[7], 512)
    spec.add(ConvBN("cnv7", feats["cnv6b"], cnv7, 512, 3, 2, decay=decay))
    cnv7b = spec.dense("cnv7b", hs[7], ws[7], 512)
    spec.add(ConvBN("cnv7b", cnv7, cnv7b, 512, 3, 1, decay=decay))
    # second placement of the shared skips; placed before both decoders so that, in the reverse
    # schedule, the decoders' full-buffer gradient writes precede the copies' slice accumulations
    for name, slot in fd.skip_slots(4).items():
        spec.add(Copy(feats[name], slot))
    disps = build_decoder(spec, dd, feats, cnv7b, H, W, hs, ws, decay, 1, 1, 10.0, 0.001)
    flows = build_decoder(spec, fd, feats, cnv7b, H, W, hs, ws, decay, 2, 0, 1.0, 0.0, icnv6_name="icnv6_opt_opt")
    spec.outputs = disps + flows
    spec.end_points = feats
    return spec
