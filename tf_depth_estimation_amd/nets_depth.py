"""MI355X-native `nets_depth` (reference: nets_depth.py): joint depth + optical-flow `disp_net` with a
shared encoder, a depth decoder (DISP_SCALING*sigmoid + MIN_DISP) and a 2-channel linear flow decoder.

    disp_net(tgt_image, is_training=True)
        -> ([disp1, disp2, disp3, disp4, flow1, flow2, flow3, flow4], end_points)   (:76-199)
"""
from . import _api, _netlib

DISP_SCALING = 10    # :8
MIN_DISP = 0.001     # :9


def disp_net(tgt_image, is_training=True):
    outs, prog = _api.run_net("depth_net", _netlib.depthflow_net_spec, tgt_image, is_training)
    return outs, {"program": prog}
