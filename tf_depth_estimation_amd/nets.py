"""MI355X-native `nets` (reference: nets.py, the original SfMLearner-style module; used by refine_depth.py:16,170).

    disp_net(tgt_image, is_training=True) -> ([disp1, disp2, disp3, disp4], end_points)        (:76-147)

Same encoder / skip decoder as nets_optflow_depth.disp_net, but the four disparity heads are 3-channel
LINEAR convs (`activation_fn=None, normalizer_fn=None`, :122-144: no sigmoid, no DISP_SCALING / MIN_DISP
applied), the bilinear up-samplings carry 3 channels (concats 64+64+3, 32+32+3, 16+3), and slim's default
BN decay 0.999 applies (batch_norm_params = {'is_training': ...}, :77).  Variables live under the enclosing
`variables.variable_scope` + 'depth_net' (:80).
"""
from . import _api, _netlib

DISP_SCALING = 10    # :8 (declared, unused by disp_net)
MIN_DISP = 0.01      # :9 (declared, unused by disp_net)


def disp_net(tgt_image, is_training=True):
    outs, prog = _api.run_net("depth_net", _netlib.disp_net_spec, tgt_image, is_training,
                              decay=0.999, head_ch=3, head_act=0)
    return outs, {"program": prog}
