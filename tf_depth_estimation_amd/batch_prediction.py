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
  * `restore(prefix)` reads the TF-1 V2 bundle (checkpoint.Saver) and re-folds/re-captures.

The host-side post-processing of batch_prediction.py:72-75 (cv2.resize INTER_CUBIC to the output size,
cv2.bilateralFilter, .tofile) stays on the host with the caller: it is OpenCV, outside the GPU path.
"""
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


class Predictor:
    """`pred = Predictor("disp_net", 224, 224)(images)` -- the sess.run(pred_disp, feed_dict=...) loop of
    batch_prediction.py with the network compiled once for a fixed (batch, H, W).

    Outputs are the reference's lists (disp_net: [disp1..disp4]; depthflow_net: [disp1..4, flow1..4];
    depth_net: [disp3, disp4, pose [b,1,6], mask3, mask4]) as views of device buffers that the next call
    overwrites (clone to keep).  Variables come from the process variable store under `scope`, so a
    network trained in this process predicts directly; `restore()` loads a checkpoint instead."""

    def __init__(self, net="disp_net", H=224, W=224, batch=1, scope="model", fold_bn=True, graph=True):
        if net not in NETS:
            raise ValueError(f"unknown net {net!r}: one of {sorted(NETS)}")
        net_scope, builder, cin, kw, _ = NETS[net]
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
