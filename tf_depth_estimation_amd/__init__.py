"""MI355X-native hot path of wrlife/tf_depth_estimation.

Reference-named modules (drop-in call signatures, output lists and TF variable names):
  nets_optflow_depth, nets_optflow_depth_pairtest, nets_depth  -- the encoder/decoder networks
  variables                                                   -- variable_scope / checkpoint contract
  losses, train                                               -- per-config fused loss heads and steps
All compute runs in libtde.so (HIP, gfx950) through the C ABI of include/tde.h; there is no CPU path.
"""
__all__ = ["nets_optflow_depth", "nets_optflow_depth_pairtest", "nets_depth", "variables"]
