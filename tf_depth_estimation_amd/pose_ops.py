"""Small pose-head ops on the GPU (HIP kernels from libtde.so)."""
import torch

from . import _lib
from ._lib import ptr


class _SpatialMean(torch.autograd.Function):
    """tf.reduce_mean(pose_pred, [1, 2]) (nets_optflow_depth.py:183)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty((N, C), device=x.device, dtype=torch.float32)
        _lib.call("tde_spatial_mean_fwd", N, H * W, C, ptr(x), C, ptr(y), _lib.stream_ptr())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        dx = torch.empty((N, H, W, C), device=dy.device, dtype=torch.float32)
        dy = dy.contiguous()
        _lib.call("tde_spatial_mean_bwd", N, H * W, C, ptr(dx), C, 0, ptr(dy), _lib.stream_ptr())
        return dx


def reduce_mean_hw(x):
    return _SpatialMean.apply(x)
