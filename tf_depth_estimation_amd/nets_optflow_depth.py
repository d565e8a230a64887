"""MI355X-native `nets_optflow_depth` (reference: nets_optflow_depth.py) -- same call signatures,
output lists and variable names; every layer runs as HIP kernels from libtde.so.

    disp_net(tgt_image, is_training=True) -> ([disp1, disp2, disp3, disp4], end_points)   (:76-147)
    depth_net(tgt_image, is_training=True) -> ([disp3, disp4], pose[b,1,6], [mask3, mask4], end_points)
                                                                                        (:151-276)
Variables are created under the enclosing `variables.variable_scope` + 'depth_net' /
'depth_cam_net', e.g. `model_singledepth/depth_net/cnv1/weights`.
"""
from . import _api, _netlib, pose_ops

DISP_SCALING = 4     # :8
MIN_DISP = 0         # :9


def disp_net(tgt_image, is_training=True):
    outs, prog = _api.run_net("depth_net", _netlib.disp_net_spec, tgt_image, is_training,
                              decay=0.99, scale=float(DISP_SCALING), offset=float(MIN_DISP))
    return outs, {"program": prog}


def depth_net(tgt_image, is_training=True):
    outs, prog = _api.run_net("depth_cam_net", _netlib.depth_net_spec, tgt_image, is_training, levels=2)
    disps, pose_pred, masks = outs[:2], outs[2], outs[3:]
    pose_final = pose_ops.reduce_mean_hw(pose_pred).reshape(-1, 1, 6)   # no 0.01 scale (:183-186)
    return disps, pose_final, masks, {"program": prog}
