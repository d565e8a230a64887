"""MI355X-native inference path of the reference's prediction scripts.

batch_prediction.py:38-75 builds `disp_net(x, is_training=False)` under variable_scope("model"),
restores a tf.train.Saver checkpoint (:49-55) and then runs `sess.run(pred_disp, feed_dict={x: I})`
once per image (batch 1, 224x224 after cv2.resize).  batch_prediction_optflow.py does the same with
nets_depth.disp_net (disparities + flows), batch_prediction_cam_est.py with depth_net (disparities,
pose, masks).  Here:

  * the inference graph is a static schedule of C-ABI calls (program.NetProgram) whose every
    conv/deconv + BatchNorm(moving statistics) + ReLU is ONE bias+ReLU conv launch on weights with the
    BN folded in (tde_bn_fold, tde_conv2d_fwd_bias_act / tde_deconv2d_fwd_bias_act) -- no pre-BN tensor,
    no separate normalisation pass;
  * the whole forward is captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed per call,
    so a batch-1 prediction is one graph launch (latency-bound at batch 1: ~30 layers);
  * `restore(prefix)` reads the TF-1 V2 bundle (checkpoint.Saver) and re-folds/re-captures;
  * the script's OpenCV steps run on the GPU too (csrc/postproc.hip, restated from OpenCV's published scalar
    code -- cv2 is not vendored, parity unpinned): `resize_area` for `cv2.resize(I, (224, 224), INTER_AREA)` (:62),
    written straight into the network input, `resize_cubic` + `bilateral_filter` for
    `cv2.resize(pred[0][0,:,:,0], (image_width, image_height), INTER_CUBIC)` and `cv2.bilateralFilter(z, 9, 75, 75)`
    (:72-73); `Predictor.predict_depth_map` is the loop body of batch_prediction.py:58-75 (uint8 image -> z map).
"""
import ctypes

import torch

from . import _api, _lib, _netlib, checkpoint, pose_ops, variables
from .program import NetRun

# net name -> (variable scope of the net, spec builder, input channels, builder kwargs, reference)
NETS = {
    "disp_net": ("depth_net", _netlib.disp_net_spec, 3, dict(decay=0.99, scale=4.0, offset=0.0),
                 "nets_optflow_depth.disp_net (batch_prediction.py:41-44)"),
    "depthflow_net": ("depth_net", _netlib.depthflow_net_spec, 6, {},
                      "nets_depth.disp_net (batch_prediction_optflow.py)"),
    "depth_net": ("depth_cam_net", _netlib.depth_net_spec, 6, dict(levels=2),
                  "nets_optflow_depth.depth_net (batch_prediction_cam_est.py)"),
}


def resize_area(images, oh, ow, out=None, out_f32=None):
    """cv2.resize(I, (ow, oh), interpolation=cv2.INTER_AREA) (batch_prediction.py:62) of a uint8 [B,H,W,C] device
    batch (C <= 4) -> uint8 [B,oh,ow,C] (`out`), and / or its float values into `out_f32` ([B,oh,ow,>=C], e.g. a
    network input).  Returns `out` (allocated when neither output is given)."""
    if images.dtype != torch.uint8 or images.dim() != 4 or not images.is_contiguous():
        raise ValueError("resize_area expects a contiguous uint8 [B,H,W,C] tensor")
    B, H, W, C = images.shape
    if out is None and out_f32 is None:
        out = torch.empty((B, oh, ow, C), dtype=torch.uint8, device=images.device)
    fcs = 0
    if out_f32 is not None:
        if out_f32.dtype != torch.float32 or tuple(out_f32.shape[:3]) != (B, oh, ow) or out_f32.shape[3] < C:
            raise ValueError("out_f32 must be float32 [B,oh,ow,>=C]")
        fcs = out_f32.stride(2)
        if out_f32.stride(1) != ow * fcs or out_f32.stride(0) != oh * ow * fcs:
            raise ValueError("out_f32 must be a pixel-major channel view")
    if out is not None and (tuple(out.shape) != (B, oh, ow, C) or out.dtype != torch.uint8 or not out.is_contiguous()):
        raise ValueError("out must be a contiguous uint8 [B,oh,ow,C] tensor")
    lib = _lib.load()
    _lib.check(lib.tde_resize_area_u8(B, H, W, C, _lib.ptr(images), oh, ow, _lib.ptr(out), _lib.ptr(out_f32), fcs,
                                      _lib.stream_ptr()), "resize_area")
    return out


def resize_cubic(maps, oh, ow, out=None):
    """cv2.resize(z, (ow, oh), interpolation=cv2.INTER_CUBIC) (batch_prediction.py:72) of a float [B,H,W] batch or
    of channel 0 of a [B,H,W,C] view (e.g. a disparity output) -> float [B,oh,ow]."""
    if maps.dtype != torch.float32:
        raise ValueError("resize_cubic expects float32 maps")
    t = maps if maps.dim() == 4 else maps.unsqueeze(-1)
    B, H, W, _ = t.shape
    cs = t.stride(2)
    if t.stride(1) != W * cs or t.stride(0) != H * W * cs:
        raise ValueError("resize_cubic expects a pixel-major [B,H,W(,C)] view")
    if out is None:
        out = torch.empty((B, oh, ow), dtype=torch.float32, device=maps.device)
    lib = _lib.load()
    _lib.check(lib.tde_resize_cubic_f32(B, H, W, _lib.ptr(t), cs, 0, oh, ow, _lib.ptr(out), _lib.stream_ptr()),
               "resize_cubic")
    return out


_BIL_WS = {}


def bilateral_filter(maps, d=9, sigma_color=75.0, sigma_space=75.0, out=None):
    """cv2.bilateralFilter(z, d, sigma_color, sigma_space) (batch_prediction.py:73) of each map of a dense float
    [B,H,W] batch (BORDER_REFLECT_101) -> float [B,H,W]."""
    if maps.dtype != torch.float32 or maps.dim() != 3 or not maps.is_contiguous():
        raise ValueError("bilateral_filter expects a contiguous float32 [B,H,W] tensor")
    B, H, W = maps.shape
    if out is None:
        out = torch.empty_like(maps)
    lib = _lib.load()
    nb = lib.tde_bilateral_workspace_size(B)
    ws = _BIL_WS.get((maps.device, B))
    if ws is None:
        ws = _BIL_WS[(maps.device, B)] = torch.empty(max(nb // 4, 4), dtype=torch.float32, device=maps.device)
    _lib.check(lib.tde_bilateral_f32(B, H, W, _lib.ptr(maps), _lib.ptr(out), int(d), ctypes.c_double(sigma_color),
                                     ctypes.c_double(sigma_space), _lib.ptr(ws), nb, _lib.stream_ptr()),
               "bilateral_filter")
    return out


class Predictor:
    """`pred = Predictor("disp_net", 224, 224)(images)` -- the sess.run(pred_disp, feed_dict=...) loop of
    batch_prediction.py with the network compiled once for a fixed (batch, H, W).

    Outputs are the reference's lists (disp_net: [disp1..disp4]; depthflow_net: [disp1..4, flow1..4];
    depth_net: [disp3, disp4, pose [b,1,6], mask3, mask4]) as views of device buffers that the next call
    overwrites (clone to keep).  Variables come from the process variable store under `scope`, so a
    network trained in this process predicts directly; `restore()` loads a checkpoint instead."""

    def __init__(self, net="disp_net", H=224, W=224, batch=1, scope="model", fold_bn=True, graph=True, cin=None):
        """cin: input channels when not the net's usual count -- batch_prediction_optflow.py:43 feeds depth_net an
        11-channel [I, I1, flow, I_warp] stack at 240x720."""
        if net not in NETS:
            raise ValueError(f"unknown net {net!r}: one of {sorted(NETS)}")
        net_scope, builder, cin0, kw, _ = NETS[net]
        cin = cin0 if cin is None else int(cin)
        self.net, self.fold, self.use_graph = net, bool(fold_bn), bool(graph)
        with variables.variable_scope(scope):
            self.prog = _api.get_program(net_scope, builder, H, W, cin, **kw)
        self.run = NetRun(self.prog, batch)
        self.x = torch.zeros((batch, H, W, cin), dtype=torch.float32, device="cuda")
        self.outs = None
        self.graph = None
        self.refresh()

    def _forward(self):
        outs = self.prog.forward(self.run, self.x, is_training=False, fold_bn=self.fold)
        if self.net == "depth_net":
            disps, pose_pred, masks = outs[:2], outs[2], outs[3:]
            outs = disps + [pose_ops.reduce_mean_hw(pose_pred).reshape(-1, 1, 6)] + masks   # :183-186
        return outs

    def refresh(self):
        """Re-fold the BN statistics and re-capture after the variables changed."""
        self.graph = None
        if self.fold:
            self.prog.fold_bn()
        s = _lib.owned_stream(self, "warmup")
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):               # warm-up: allocates every lazily created buffer
            self.outs = self._forward()
        torch.cuda.current_stream().wait_stream(s)
        if self.use_graph:
            g = torch.cuda.CUDAGraph()
            with _lib.capture_scope(), torch.cuda.graph(g, stream=_lib.owned_stream(self, "capture"),
                                                        capture_error_mode="thread_local"):
                self.outs = self._forward()
            self.graph = g

    def restore(self, save_path):
        """saver.restore(sess, checkpoint) (batch_prediction.py:55), then re-fold / re-capture."""
        checkpoint.Saver().restore(None, save_path)
        self.refresh()

    def predict_depth_map(self, image_u8, out_hw=(240, 720)):
        """The body of batch_prediction.py:58-75 for one decoded image (uint8 [h,w,3] or a [B,h,w,3] batch, host or
        device): INTER_AREA resize into the network input (:62; the pixel values 0..255 are fed as they are -- the
        script's /255 is commented out, :65-67), the prediction (:70), then the INTER_CUBIC resize of disp1's map to
        out_hw = (FLAGS.image_height, FLAGS.image_width) (:72) and the 9 / 75 / 75 bilateral filter (:73).  Returns
        the float [B, out_h, out_w] maps the script writes with .tofile (:75)."""
        if self.net != "disp_net":
            raise ValueError("predict_depth_map is batch_prediction.py's disp_net path")
        img = image_u8 if image_u8.dim() == 4 else image_u8.unsqueeze(0)
        img = img.to(device=self.x.device, dtype=torch.uint8).contiguous()
        B, H, W = self.x.shape[:3]
        if img.shape[0] != B or img.shape[3] != 3:
            raise ValueError(f"expected {B} RGB image(s), got {tuple(img.shape)}")
        resize_area(img, H, W, out_f32=self.x)
        if self.graph is not None:
            self.graph.replay()
        else:
            self.outs = self._forward()
        z = resize_cubic(self.outs[0], out_hw[0], out_hw[1])
        return bilateral_filter(z, 9, 75.0, 75.0)

    def predict_pose(self, image_a_u8, image_b_u8):
        """The loop body of batch_prediction_cam_est.py:79-98: both decoded images INTER_AREA-resized (:82,88) straight
        into the two channel halves of the network input (the concat of :90), the depth_net prediction, and the pose
        [B, 6] the script saves with np.savetxt (:98)."""
        if self.net != "depth_net" or self.x.shape[3] != 6:
            raise ValueError("predict_pose is batch_prediction_cam_est.py's 6-channel depth_net path")
        B, H, W = self.x.shape[:3]
        for half, img in ((0, image_a_u8), (1, image_b_u8)):
            t = img if img.dim() == 4 else img.unsqueeze(0)
            t = t.to(device=self.x.device, dtype=torch.uint8).contiguous()
            if t.shape[0] != B or t.shape[3] != 3:
                raise ValueError(f"expected {B} RGB image(s), got {tuple(t.shape)}")
            resize_area(t, H, W, out_f32=self.x[..., 3 * half:3 * half + 3])
        if self.graph is not None:
            self.graph.replay()
        else:
            self.outs = self._forward()
        return self.outs[2].reshape(B, 6)

    def __call__(self, images):
        """images: [batch, H, W, cin] float32 (host or device).  Returns the output list."""
        if tuple(images.shape) != tuple(self.x.shape):
            raise ValueError(f"expected input {tuple(self.x.shape)}, got {tuple(images.shape)}")
        self.x.copy_(images, non_blocking=True)
        if self.graph is not None:
            self.graph.replay()
        else:
            self.outs = self._forward()
        return self.outs
