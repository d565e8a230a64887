"""TEST INFRASTRUCTURE ONLY -- NumPy restatement of the three OpenCV calls of the reference's prediction script
(batch_prediction.py:62,72-73), the checker of csrc/postproc.hip.  Only tests/ may import it.

    I = cv2.resize(I, (224, 224), interpolation=cv2.INTER_AREA)                          -> resize_area_u8
    z = cv2.resize(pred[0][0,:,:,0], (image_width, image_height), interpolation=cv2.INTER_CUBIC)  -> resize_cubic
    z = cv2.bilateralFilter(z, 9, 75, 75)                                                -> bilateral

OpenCV is a pip dependency of the reference (`import cv2`, no version pinned, nothing vendored) and is not
importable here, so these restate OpenCV 4.x's published scalar reference code (modules/imgproc/src/resize.cpp:
cv::resize -> hal::resize, resizeAreaFast_, computeResizeAreaTab + ResizeArea_Invoker, resizeGeneric_ with
interpolateCubic / area-mode linear coefficients; bilateral_filter.simd.hpp bilateralFilter_32f): PARITY UNPINNED
against cv2 itself.  Known divergence of OpenCV's own builds from its scalar code: on x86 the 8-bit 2x2 area
average and the 8-bit linear vertical pass run SIMD code that rounds half up instead of to nearest even; the scalar
semantics are restated.  float32 arithmetic in OpenCV's operation order (multiply, then add; no fused multiply-add).
"""
import math

import numpy as np

F = np.float32
FLT_EPSILON = float(np.finfo(np.float32).eps)
DBL_EPSILON = float(np.finfo(np.float64).eps)


def _round_half_even_u8(v):
    """saturate_cast<uchar>(float): cvRound (nearest, ties to even), then clamp to [0, 255]."""
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def _area_tab(ssize, dsize, scale):
    """computeResizeAreaTab: per destination index the (source index, weight) list, in table order."""
    out = []
    for d in range(dsize):
        fs1 = d * scale
        fs2 = fs1 + scale
        cell = min(scale, ssize - fs1)
        s1, s2 = math.ceil(fs1), math.floor(fs2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        taps = []
        if s1 - fs1 > 1e-3:
            taps.append((s1 - 1, F((s1 - fs1) / cell)))
        for s in range(s1, s2):
            taps.append((s, F(1.0 / cell)))
        if fs2 - s2 > 1e-3:
            taps.append((s2, F(min(min(fs2 - s2, 1.0), cell) / cell)))
        out.append(taps)
    return out


def resize_area_u8(img, oh, ow):
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_AREA) for uint8 [H, W, C] (resize.cpp)."""
    img = np.asarray(img, np.uint8)
    H, W, C = img.shape
    if (H, W) == (oh, ow):
        return img.copy()
    inv_x, inv_y = ow / W, oh / H            # cv::resize: inv_scale = dsize / ssize
    sx, sy = 1.0 / inv_x, 1.0 / inv_y        # hal::resize: scale = 1 / inv_scale
    ix, iy = int(round(sx)), int(round(sy))
    fast = abs(sx - ix) < DBL_EPSILON and abs(sy - iy) < DBL_EPSILON
    out = np.zeros((oh, ow, C), np.uint8)
    if sx >= 1 and sy >= 1:
        if fast:
            # resizeAreaFast_ (scalar): int sum of the cell * (1.f / area), rounded; edge cells: sum / count
            scale = F(F(1.0) / F(ix * iy))
            for dy in range(oh):
                for dx in range(ow):
                    cell = img[dy * iy:min(dy * iy + iy, H), dx * ix:min(dx * ix + ix, W)].astype(np.int64)
                    s = cell.reshape(-1, C).sum(0)
                    if dy * iy + iy <= H and dx < W // ix:
                        out[dy, dx] = _round_half_even_u8(s.astype(F) * scale)
                    else:
                        n = cell.shape[0] * cell.shape[1]
                        out[dy, dx] = _round_half_even_u8(s.astype(F) / F(n)) if n else 0
            return out
        # ResizeArea_Invoker: buf = sum_x S*alpha (float, table order), sum = beta_0*buf_0 (+ beta_j*buf_j)
        xt, yt = _area_tab(W, ow, sx), _area_tab(H, oh, sy)
        imf = img.astype(F)
        for dy in range(oh):
            acc = None
            for j, (s_y, beta) in enumerate(yt[dy]):
                row = imf[s_y]
                buf = np.zeros((ow, C), F)
                for dx in range(ow):
                    b = np.zeros(C, F)
                    for s_x, alpha in xt[dx]:
                        b = (b + row[s_x] * alpha).astype(F)
                    buf[dx] = b
                term = (F(beta) * buf).astype(F)
                acc = term if j == 0 else (acc + term).astype(F)
            out[dy] = _round_half_even_u8(acc)
        return out
    # area-mode emulation by 8-bit fixed-point linear interpolation (resizeGeneric_, INTER_RESIZE_COEF_BITS 11)
    xs = []
    for dx in range(ow):
        s = math.floor(dx * sx)
        f = F((dx + 1) - (s + 1) * inv_x)
        f = F(0) if f <= 0 else F(f - F(math.floor(f)))
        if s < 0:
            f, s = F(0), 0
        hi = s + 1 >= W
        if s >= W - 1:
            f, s = F(0), W - 1
        xs.append((s, int(np.rint(F(F(1) - f) * F(2048))), int(np.rint(f * F(2048))), hi))
    out = np.zeros((oh, ow, C), np.uint8)
    im = img.astype(np.int64)
    for dy in range(oh):
        s = math.floor(dy * sy)
        f = F((dy + 1) - (s + 1) * inv_y)
        f = F(0) if f <= 0 else F(f - F(math.floor(f)))
        b0, b1 = int(np.rint(F(F(1) - f) * F(2048))), int(np.rint(f * F(2048)))
        rows = [im[min(max(s + k, 0), H - 1)] for k in range(2)]
        for dx, (x0, a0, a1, hi) in enumerate(xs):
            v = [r[x0] * 2048 if hi else r[x0] * a0 + r[x0 + 1] * a1 for r in rows]
            out[dy, dx] = np.clip((v[0] * b0 + v[1] * b1 + (1 << 21)) >> 22, 0, 255)
    return out


def _cubic_coeffs(x):
    """interpolateCubic, A = -0.75, float arithmetic:
    c0 = ((A*(x + 1) - 5*A)*(x + 1) + 8*A)*(x + 1) - 4*A, c1 = ((A + 2)*x - (A + 3))*x*x + 1,
    c2 = ((A + 2)*(1 - x) - (A + 3))*(1 - x)*(1 - x) + 1, c3 = 1 - c0 - c1 - c2."""
    A, one, x = F(-0.75), F(1), F(x)
    xp = F(x + one)
    t = F(A * xp)
    t = F(t - F(F(5) * A))
    t = F(t * xp)
    t = F(t + F(F(8) * A))
    t = F(t * xp)
    c0 = F(t - F(F(4) * A))

    def mid(u):
        t = F(F(A + F(2)) * u)
        t = F(t - F(A + F(3)))
        t = F(t * u)
        t = F(t * u)
        return F(t + one)
    c1 = mid(x)
    c2 = mid(F(one - x))
    c3 = F(F(F(one - c0) - c1) - c2)
    return [c0, c1, c2, c3]


def resize_cubic(src, oh, ow):
    """cv2.resize(src, (ow, oh), interpolation=cv2.INTER_CUBIC) for a float32 [H, W] map (resize.cpp)."""
    src = np.asarray(src, F)
    H, W = src.shape
    if (H, W) == (oh, ow):
        return src.copy()
    sx, sy = 1.0 / (ow / W), 1.0 / (oh / H)

    def taps(d, scale, n):
        f = F((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = F(f - F(s))
        return [min(max(s - 1 + k, 0), n - 1) for k in range(4)], _cubic_coeffs(f)
    xt = [taps(dx, sx, W) for dx in range(ow)]
    xi = np.array([t[0] for t in xt])              # [ow, 4]
    xc = np.array([t[1] for t in xt], F)           # [ow, 4]
    out = np.zeros((oh, ow), F)
    for dy in range(oh):
        ys, cy = taps(dy, sy, H)
        rows = []
        for k in range(4):
            r = src[ys[k]][xi]                     # [ow, 4]
            v = np.zeros(ow, F)
            for j in range(4):
                v = (v + (r[:, j] * xc[:, j]).astype(F)).astype(F)
            rows.append(v)
        acc = (cy[0] * rows[0]).astype(F)
        for k in range(1, 4):
            acc = (acc + (cy[k] * rows[k]).astype(F)).astype(F)
        out[dy] = acc
    return out


def bilateral(src, d=9, sigma_color=75.0, sigma_space=75.0):
    """cv2.bilateralFilter(src, d, sigma_color, sigma_space) for a float32 [H, W] map (bilateralFilter_32f, one
    channel, BORDER_REFLECT_101)."""
    src = np.asarray(src, F)
    H, W = src.shape
    if sigma_color <= 0:
        sigma_color = 1.0
    if sigma_space <= 0:
        sigma_space = 1.0
    gc = -0.5 / (sigma_color * sigma_color)
    gs = -0.5 / (sigma_space * sigma_space)
    radius = int(round(sigma_space * 1.5)) if d <= 0 else d // 2
    radius = max(radius, 1)
    fin = src[~np.isnan(src)]
    lo, hi = float(fin.min()), float(fin.max())
    if abs(lo - hi) < FLT_EPSILON:
        return src.copy()
    nbins = 1 << 12
    length = F(hi - lo)
    scale_index = F(F(nbins) / length)
    lut = np.array([F(math.exp(float(F(F(i) / scale_index)) ** 2 * gc)) for i in range(nbins + 2)], F)
    taps = []
    for i in range(-radius, radius + 1):
        for j in range(-radius, radius + 1):
            r = math.sqrt(float(i) * i + float(j) * j)
            if r > radius or (i == 0 and j == 0):
                continue
            taps.append((i, j, F(math.exp(r * r * gs))))
    pad = np.pad(src, radius, mode="reflect")     # numpy "reflect" = BORDER_REFLECT_101
    s = np.zeros((H, W), F)
    ws = np.zeros((H, W), F)
    rval = src
    nan_r = np.isnan(rval)
    for i, j, w_sp in taps:
        val = pad[radius + i:radius + i + H, radius + j:radius + j + W]
        alpha = (np.abs((val - rval).astype(F)) * scale_index).astype(F)
        ok = ~np.isnan(val)
        idx = np.zeros((H, W), np.int64)
        idx[ok] = np.floor(alpha[ok]).astype(np.int64)
        alpha = (alpha - idx.astype(F)).astype(F)
        li = lut[np.clip(idx, 0, nbins)]
        li1 = lut[np.clip(idx + 1, 0, nbins + 1)]
        cw = (li + (alpha * (li1 - li).astype(F)).astype(F)).astype(F)
        w = (w_sp * np.where(nan_r, F(1), cw)).astype(F)
        ws = np.where(ok, (ws + w).astype(F), ws)
        s = np.where(ok, (s + (val * w).astype(F)).astype(F), s)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = np.where(nan_r, s / ws, (s + rval).astype(F) / (ws + F(1)).astype(F)).astype(F)
    return out
