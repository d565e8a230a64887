"""MI355X-native `nets_optflow_depth_pairtest` (reference: nets_optflow_depth_pairtest.py): the
4-scale `depth_net` whose outputs match the 4-scale loss loop of train_depth_then_cam_lr.py:211
(SURVEY.md Appendix C, config 4).

    disp_net(tgt_image, is_training=True) -> ([disp1..disp4], end_points)    (:76-147)
    depth_net(tgt_image, is_training=True)
        -> ([disp1..disp4], pose[b,1,6], [mask1..mask4], end_points)      (:151-276)
disp_net here is BN-FREE: the normalizer is commented out (:83-84), so every conv / conv2d_transpose is
slim's conv + bias + ReLU (`is_training` has no effect); heads are DISP_SCALING * sigmoid (:122-144).
depth_net's BN uses slim's default decay 0.999 (:152).
"""
from . import _api, _netlib, pose_ops

DISP_SCALING = 4
MIN_DISP = 0


def disp_net(tgt_image, is_training=True):
    outs, prog = _api.run_net("depth_net", _netlib.disp_net_spec, tgt_image, is_training, bn=False,
                              scale=float(DISP_SCALING), offset=float(MIN_DISP))
    return outs, {"program": prog}


def depth_net(tgt_image, is_training=True):
    outs, prog = _api.run_net("depth_cam_net", _netlib.depth_net_spec, tgt_image, is_training, levels=4)
    disps, pose_pred, masks = outs[:4], outs[4], outs[5:]
    pose_final = pose_ops.reduce_mean_hw(pose_pred).reshape(-1, 1, 6)
    return disps, pose_final, masks, {"program": prog}
