"""Oracle restatement of utils_lr.py / utils.py geometry and warping (TEST INFRASTRUCTURE ONLY).

Differentiable PyTorch-CPU code following the TF graph op by op, so autograd reproduces TF's
gradients: floor() has zero gradient, the out-of-range masks are constants, gathers back-propagate
as scatter-adds into the sampled image (utils_lr.py:276-366).
"""
import torch


def axis_angle_to_rotation_matrix(axis, angle):
    """utils_lr.py:77-103: R = I + sin(a)[u]x + (1-cos(a))[u]x^2 with M built from (ux,uy,uz)."""
    B = axis.shape[0]
    z = torch.zeros(B, dtype=axis.dtype)
    ax, ay, az = axis[:, 0], axis[:, 1], axis[:, 2]
    # M = [[0,-az,ay],[0,0,-ax],[0,0,0]]; cp = M - M^T (utils_lr.py:85-91)
    M = torch.stack([torch.stack([z, -az, ay], -1),
                     torch.stack([z, z, -ax], -1),
                     torch.stack([z, z, z], -1)], 1)
    cp = M - M.transpose(1, 2)
    eye = torch.eye(3, dtype=axis.dtype).expand(B, 3, 3)
    return eye + torch.sin(angle) * cp + (1 - torch.cos(angle)) * (cp @ cp)


def euler2mat(z, y, x):
    """utils_lr.py:26-75 (R = Rx @ Ry @ Rz) with the angles clipped to [-pi, pi]."""
    import math
    z = z.clamp(-math.pi, math.pi).reshape(-1)
    y = y.clamp(-math.pi, math.pi).reshape(-1)
    x = x.clamp(-math.pi, math.pi).reshape(-1)
    o, n = torch.ones_like(z), torch.zeros_like(z)
    zm = torch.stack([torch.stack([z.cos(), -z.sin(), n], -1), torch.stack([z.sin(), z.cos(), n], -1),
                      torch.stack([n, n, o], -1)], 1)
    ym = torch.stack([torch.stack([y.cos(), n, y.sin()], -1), torch.stack([n, o, n], -1),
                      torch.stack([-y.sin(), n, y.cos()], -1)], 1)
    xm = torch.stack([torch.stack([o, n, n], -1), torch.stack([n, x.cos(), -x.sin()], -1),
                      torch.stack([n, x.sin(), x.cos()], -1)], 1)
    return xm @ ym @ zm


def pose_vec2mat(vec, format="angleaxis"):
    """utils_lr.py:106-149: [B,6] (tx,ty,tz,rx,ry,rz) -> [B,4,4].  angleaxis: angle = ||r||,
    axis = r/angle (NaN at r = 0, as in the reference)."""
    B = vec.shape[0]
    t = vec[:, 0:3].unsqueeze(-1)
    if format == "angleaxis":
        r = vec[:, 3:6]
        angle = torch.linalg.norm(r, dim=1, keepdim=True)
        axis = r / angle
        rot = axis_angle_to_rotation_matrix(axis, angle.unsqueeze(-1))
    elif format == "eular":
        rot = euler2mat(vec[:, 5], vec[:, 4], vec[:, 3])
    else:
        raise ValueError(format)
    filler = torch.tensor([0.0, 0.0, 0.0, 1.0], dtype=vec.dtype).reshape(1, 1, 4).expand(B, 1, 4)
    return torch.cat([torch.cat([rot, t], 2), filler], 1)


def meshgrid(batch, height, width, dtype=torch.float64, homogeneous=True):
    """utils_lr.py:196-220: x = (linspace(-1,1,W)+1)*0.5*(W-1) -> [B, 3 (or 2), H, W]."""
    xs = (torch.linspace(-1.0, 1.0, width, dtype=dtype) + 1.0) * 0.5 * (width - 1)
    ys = (torch.linspace(-1.0, 1.0, height, dtype=dtype) + 1.0) * 0.5 * (height - 1)
    xt = xs.view(1, width).expand(height, width)
    yt = ys.view(height, 1).expand(height, width)
    parts = [xt, yt] + ([torch.ones_like(xt)] if homogeneous else [])
    return torch.stack(parts, 0).unsqueeze(0).expand(batch, -1, -1, -1)


def pixel2cam(depth, pixel_coords, intrinsics):
    """utils_lr.py:151-170: K^-1 [u,v,1]^T * depth, homogeneous -> [B,4,H,W]."""
    B, H, W = depth.shape
    pc = pixel_coords.reshape(B, 3, -1)
    cam = torch.linalg.inv(intrinsics) @ pc * depth.reshape(B, 1, -1)
    cam = torch.cat([cam, torch.ones(B, 1, H * W, dtype=depth.dtype)], 1)
    return cam.reshape(B, 4, H, W)


def cam2pixel(cam_coords, proj):
    """utils_lr.py:172-194: p = proj @ X; (x/(z+1e-10), y/(z+1e-10)) -> [B,H,W,2] and z [B,H,W,1]."""
    B, _, H, W = cam_coords.shape
    u = proj @ cam_coords.reshape(B, 4, -1)
    xu, yu, zu = u[:, 0:1], u[:, 1:2], u[:, 2:3]
    xn = xu / (zu + 1e-10)
    yn = yu / (zu + 1e-10)
    pix = torch.cat([xn, yn], 1).reshape(B, 2, H, W).permute(0, 2, 3, 1)
    return pix, zu.reshape(B, H, W, 1)


def bilinear_sampler(imgs, coords):
    """utils_lr.py:276-366 (== utils.py:219-308): 4-tap bilinear gather; weights from the
    UNclamped x0=floor(x), x1=x0+1, a tap's weight zeroed when its index was clamped; gathers use
    clamped indices.  Returns (output [B,Ht,Wt,C], wmask = sum of the 4 weights [B,Ht,Wt,1])."""
    B, Hs, Ws, C = imgs.shape
    _, Ht, Wt, _ = coords.shape
    cx, cy = coords[..., 0:1], coords[..., 1:2]
    x0 = torch.floor(cx).detach()
    y0 = torch.floor(cy).detach()
    x1, y1 = x0 + 1, y0 + 1
    x0s, x1s = x0.clamp(0, Ws - 1), x1.clamp(0, Ws - 1)
    y0s, y1s = y0.clamp(0, Hs - 1), y1.clamp(0, Hs - 1)
    wx0 = (x1 - cx) * (x0 == x0s).to(imgs.dtype)
    wx1 = (cx - x0) * (x1 == x1s).to(imgs.dtype)
    wy0 = (y1 - cy) * (y0 == y0s).to(imgs.dtype)
    wy1 = (cy - y0) * (y1 == y1s).to(imgs.dtype)
    flat = imgs.reshape(-1, C)
    base = (torch.arange(B).view(B, 1, 1, 1) * (Hs * Ws))

    def g(yy, xx):
        idx = (base + yy.long() * Ws + xx.long()).reshape(-1)
        return flat[idx].reshape(B, Ht, Wt, C)

    w00, w01, w10, w11 = wx0 * wy0, wx0 * wy1, wx1 * wy0, wx1 * wy1
    out = w00 * g(y0s, x0s) + w01 * g(y1s, x0s) + w10 * g(y0s, x1s) + w11 * g(y1s, x1s)
    return out, w00 + w01 + w10 + w11


def projective_inverse_warp(img, depth, pose, intrinsics, format="angleaxis"):
    """utils_lr.py:222-256: returns (warped, src_pixel_coords, wmask, src_depth(z), pose4x4).
    `format='matrix'` (anything but eular/angleaxis) takes `pose` as a [B,4,4] matrix (:238-239)."""
    B, H, W, _ = img.shape
    if format in ("eular", "angleaxis"):
        pose = pose_vec2mat(pose, format)
    pix = meshgrid(B, H, W, dtype=img.dtype)
    cam = pixel2cam(depth, pix, intrinsics)
    filler = torch.tensor([0.0, 0.0, 0.0, 1.0], dtype=img.dtype).reshape(1, 1, 4).expand(B, 1, 4)
    K4 = torch.cat([torch.cat([intrinsics, torch.zeros(B, 3, 1, dtype=img.dtype)], 2), filler], 1)
    proj = K4 @ pose
    src_pix, src_depth = cam2pixel(cam, proj)
    out, wmask = bilinear_sampler(img, src_pix)
    return out, src_pix, wmask, src_depth, pose


def optflow_warp(img, flowx, flowy):
    """utils_lr.py:258-274: sample img at grid + flow."""
    B, H, W, _ = img.shape
    g = meshgrid(B, H, W, dtype=img.dtype, homogeneous=False).permute(0, 2, 3, 1)
    coords = torch.cat([g[..., 0:1] + flowx, g[..., 1:2] + flowy], -1)
    out, _ = bilinear_sampler(img, coords)
    return out


def consistent_depth_loss(src_depth, pred_src_depth, coords):
    """utils_lr.py:369-458: |pred_src_depth - bilinear(src_depth, coords)| (no wmask)."""
    out, _ = bilinear_sampler(src_depth, coords)
    return torch.abs(pred_src_depth - out)


def depth_optflow(src_pixel_coords):
    """utils_lr.py:472-489: flow = warped coords - pixel grid."""
    B, H, W, _ = src_pixel_coords.shape
    g = meshgrid(B, H, W, dtype=src_pixel_coords.dtype, homogeneous=False).permute(0, 2, 3, 1)
    return src_pixel_coords[..., 0:1] - g[..., 0:1], src_pixel_coords[..., 1:2] - g[..., 1:2]


def make_intrinsics_matrix(fx, fy, cx, cy):
    """Demon_Data_loader.py:14-23."""
    z, o = torch.zeros_like(fx), torch.ones_like(fx)
    return torch.stack([torch.stack([fx, z, cx], 1), torch.stack([z, fy, cy], 1),
                        torch.stack([z, z, o], 1)], 1)


def get_multi_scale_intrinsics(K, num_scales):
    """Demon_Data_loader.py:25-39: fx, fy, cx, cy divided by 2^s (not (c+0.5)/2^s-0.5)."""
    out = []
    for s in range(num_scales):
        f = 2.0 ** s
        out.append(make_intrinsics_matrix(K[:, 0, 0] / f, K[:, 1, 1] / f, K[:, 0, 2] / f, K[:, 1, 2] / f))
    return torch.stack(out, 1)
