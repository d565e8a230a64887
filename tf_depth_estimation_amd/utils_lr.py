"""MI355X-native `utils_lr` (reference: utils_lr.py): the geometry functions of the self-supervised loss
head under their reference names, signatures and output tuples, as differentiable ops over libtde.so.

    pose_vec2mat(vec, format)                                   -> [B,4,4]                   (:106-149)
    meshgrid(batch, height, width, is_homogeneous=True)         -> [B,3|2,H,W]               (:196-220)
    pixel2cam(depth, pixel_coords, intrinsics, is_homogeneous)  -> [B,4|3,H,W]               (:151-170)
    cam2pixel(cam_coords, proj)                                 -> ([B,H,W,2], [B,H,W,1])    (:172-194)
    projective_inverse_warp(img, depth, pose, intrinsics, format='eular')
        -> (output_img, src_pixel_coords, wmask, src_depth, pose)                            (:222-256)
    optflow_warp(img, flowx, flowy)                             -> output_img                (:258-274)
    bilinear_sampler(imgs, coords)                              -> (output, wmask)           (:276-366)
    consistent_depth_loss(src_depth, pred_src_depth, coords)    -> |pred - sampled|          (:369-458)
    depth_optflow(src_pixel_coords)                             -> (optflowx, optflowy)      (:472-489)

The training steps (train.py) never call these: they run the fused loss kernels (tde_warp_loss), which
compute the same terms and their gradients in one pass.  These are the un-fused building blocks for
callers that assemble their own loss, exactly as the reference scripts do.  The warp, sampler and pose
math runs in HIP kernels (warp_fwd / sampler_bwd / cam_coords_bwd / pose_vec2mat kernels); meshgrid,
pixel2cam and cam2pixel are tiny batched 3x3/4x4 products kept as device tensor ops.  Intrinsics are
data (no gradient), as at every reference call site.
"""
import torch

from . import _lib
from ._lib import ptr

FORMATS = {"angleaxis": 0, "eular": 1, "test": 2}


def _st():
    return _lib.stream_ptr()


def _f32(t):
    if t.dtype != torch.float32 or not t.is_cuda:
        raise TypeError("utils_lr ops take float32 CUDA tensors")
    return t.contiguous()


class _PoseVec2Mat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, vec, fmt):
        vec = _f32(vec)
        B = vec.shape[0]
        T = torch.empty((B, 4, 4), device=vec.device, dtype=torch.float32)
        _lib.call("tde_pose_vec2mat", B, ptr(vec), fmt, ptr(T), _st())
        ctx.save_for_backward(vec)
        ctx.fmt = fmt
        return T

    @staticmethod
    def backward(ctx, dT):
        (vec,) = ctx.saved_tensors
        dvec = torch.empty_like(vec)
        _lib.call("tde_pose_vec2mat_bwd", vec.shape[0], ptr(vec), ctx.fmt, ptr(dT.contiguous()), ptr(dvec), 0, _st())
        return dvec, None


def pose_vec2mat(vec, format):
    """[B,6] (tx,ty,tz,rx,ry,rz) -> [B,4,4] (utils_lr.py:106-149).  'angleaxis' is NaN at r = 0, as in the
    reference (:129-132)."""
    if format not in FORMATS:
        raise ValueError(f"unknown pose format {format!r}")
    if vec.dim() != 2 or vec.shape[1] != 6:
        raise ValueError(f"pose vector must be [B,6], got {tuple(vec.shape)}")
    return _PoseVec2Mat.apply(vec, FORMATS[format])


def meshgrid(batch, height, width, is_homogeneous=True, device="cuda"):
    """utils_lr.py:196-220: x = (linspace(-1,1,W)+1)*0.5*(W-1) (fp32, as TF), y likewise, [+ones]."""
    xs = (torch.linspace(-1.0, 1.0, width, device=device) + 1.0) * 0.5 * (width - 1)
    ys = (torch.linspace(-1.0, 1.0, height, device=device) + 1.0) * 0.5 * (height - 1)
    y, x = torch.meshgrid(ys, xs, indexing="ij")
    planes = [x, y] + ([torch.ones_like(x)] if is_homogeneous else [])
    return torch.stack(planes, 0).unsqueeze(0).expand(batch, -1, -1, -1).contiguous()


def pixel2cam(depth, pixel_coords, intrinsics, is_homogeneous=True):
    """utils_lr.py:151-170: cam = depth * K^-1 [u v 1]^T (+ ones row)."""
    B, H, W = depth.shape[:3]
    pc = pixel_coords.reshape(B, 3, H * W)
    cam = torch.linalg.inv(intrinsics) @ pc * depth.reshape(B, 1, H * W)
    if is_homogeneous:
        cam = torch.cat([cam, torch.ones_like(cam[:, :1])], 1)
    return cam.reshape(B, -1, H, W)


def cam2pixel(cam_coords, proj):
    """utils_lr.py:172-194: p = proj @ cam; (x/(z+1e-10), y/(z+1e-10)) as [B,H,W,2], and z [B,H,W,1]."""
    B, _, H, W = cam_coords.shape
    p = proj @ cam_coords.reshape(B, 4, H * W)
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    xn, yn = x / (z + 1e-10), y / (z + 1e-10)
    coords = torch.stack([xn, yn], -1).reshape(B, H, W, 2)
    return coords, z.reshape(B, H, W, 1)


class _Sampler(torch.autograd.Function):
    @staticmethod
    def forward(ctx, imgs, coords):
        imgs, coords = _f32(imgs), _f32(coords)
        B, Hs, Ws, C = imgs.shape
        Bc, H, W, two = coords.shape
        if Bc != B or two != 2:
            raise ValueError(f"bilinear_sampler: imgs {tuple(imgs.shape)} vs coords {tuple(coords.shape)}")
        out = torch.empty((B, H, W, C), device=imgs.device, dtype=torch.float32)
        wmask = torch.empty((B, H, W, 1), device=imgs.device, dtype=torch.float32)
        _lib.call("tde_warp_fwd", B, H, W, C, None, 0, None, None, ptr(coords), ptr(imgs), Hs, Ws, ptr(out), None,
                  None, None, ptr(wmask), None, _st())
        ctx.save_for_backward(imgs, coords)
        return out, wmask

    @staticmethod
    def backward(ctx, d_out, d_wmask):
        imgs, coords = ctx.saved_tensors
        B, Hs, Ws, C = imgs.shape
        _, H, W, _ = coords.shape
        d_img = torch.zeros_like(imgs) if ctx.needs_input_grad[0] else None
        d_coords = torch.empty_like(coords) if ctx.needs_input_grad[1] else None
        if d_out is not None:
            d_out = d_out.contiguous()
        if d_wmask is not None:
            d_wmask = d_wmask.contiguous()
        if d_img is not None or d_coords is not None:
            _lib.call("tde_sampler_bwd", B, H, W, C, ptr(coords), ptr(imgs), Hs, Ws, ptr(d_out), ptr(d_wmask),
                      ptr(d_img) if d_out is not None else None, ptr(d_coords), _st())
        return d_img, d_coords


def bilinear_sampler(imgs, coords):
    """TF bilinear sampler of utils_lr.py:276-366: out-of-range taps are clamped and weight-masked;
    returns (output [B,H,W,C], wmask [B,H,W,1] = sum of the tap weights)."""
    return _Sampler.apply(imgs, coords)


class _ProjCoords(torch.autograd.Function):
    """(coords, z) = cam2pixel((K4 @ T), pixel2cam(depth, meshgrid, K)) in one HIP pass."""

    @staticmethod
    def forward(ctx, depth, T, K):
        depth, T, K = _f32(depth), _f32(T), _f32(K)
        B, H, W = depth.shape
        P = torch.empty((B, 12), device=depth.device, dtype=torch.float32)
        Kinv = torch.empty((B, 9), device=depth.device, dtype=torch.float32)
        _lib.call("tde_pose_prep", B, None, ptr(T), ptr(K), None, ptr(P), ptr(Kinv), _st())
        coords = torch.empty((B, H, W, 2), device=depth.device, dtype=torch.float32)
        z = torch.empty((B, H, W, 1), device=depth.device, dtype=torch.float32)
        _lib.call("tde_warp_fwd", B, H, W, 1, ptr(depth), 0, ptr(P), ptr(Kinv), None, None, 0, 0, None, ptr(coords),
                  None, None, None, ptr(z), _st())
        ctx.save_for_backward(depth, K, P, Kinv)
        return coords, z

    @staticmethod
    def backward(ctx, d_coords, d_z):
        depth, K, P, Kinv = ctx.saved_tensors
        B, H, W = depth.shape
        d_depth = torch.empty_like(depth)
        gP = torch.zeros((B, 12), device=depth.device, dtype=torch.float64)
        _lib.call("tde_cam_coords_bwd", B, H, W, ptr(depth), ptr(P), ptr(Kinv),
                  ptr(d_coords.contiguous()) if d_coords is not None else None,
                  ptr(d_z.contiguous()) if d_z is not None else None, ptr(d_depth), 0, ptr(gP), _st())
        dT = torch.empty((B, 4, 4), device=depth.device, dtype=torch.float32)
        _lib.call("tde_pose_dp_to_dt", B, ptr(K), ptr(gP), ptr(dT), _st())
        return d_depth, dT, None


def projective_inverse_warp(img, depth, pose, intrinsics, format="eular"):
    """utils_lr.py:222-256.  img: source image [B,H,W,3]; depth: target depth [B,H,W]; pose: [B,6]
    (tx,ty,tz,rx,ry,rz) for format 'eular'/'angleaxis', else an already-built [B,4,4] matrix;
    intrinsics [B,3,3].  Returns (output_img, src_pixel_coords, wmask, src_depth, pose_4x4)."""
    if depth.dim() == 4:
        depth = depth.squeeze(-1)
    if format in ("eular", "angleaxis"):
        pose = pose_vec2mat(pose, format)
    coords, z = _ProjCoords.apply(depth, pose, intrinsics)
    out, wmask = bilinear_sampler(img, coords)
    return out, coords, wmask, z, pose


def _grid_xy(B, H, W, device):
    g = meshgrid(B, H, W, is_homogeneous=False, device=device)
    return g[:, 0].unsqueeze(-1), g[:, 1].unsqueeze(-1)


def optflow_warp(img, flowx, flowy):
    """utils_lr.py:258-274: sample img at (grid_x + flowx, grid_y + flowy); flows [B,H,W,1]."""
    B, H, W, _ = img.shape
    gx, gy = _grid_xy(B, H, W, img.device)
    coords = torch.cat([gx + flowx, gy + flowy], -1)
    out, _ = bilinear_sampler(img, coords)
    return out


def consistent_depth_loss(src_depth, pred_src_depth, coords):
    """utils_lr.py:369-458: |pred_src_depth - bilinear(src_depth, coords)| (the map, not its mean)."""
    sampled, _ = bilinear_sampler(src_depth, coords)
    return (pred_src_depth - sampled).abs()


def depth_optflow(src_pixel_coords):
    """utils_lr.py:472-489: flow from the projected coordinates: coords - grid, as ([B,H,W,1], [B,H,W,1])."""
    B, H, W, _ = src_pixel_coords.shape
    gx, gy = _grid_xy(B, H, W, src_pixel_coords.device)
    return src_pixel_coords[..., 0:1] - gx, src_pixel_coords[..., 1:2] - gy


__all__ = ["pose_vec2mat", "meshgrid", "pixel2cam", "cam2pixel", "projective_inverse_warp", "optflow_warp",
           "bilinear_sampler", "consistent_depth_loss", "depth_optflow"]
