"""Pure NumPy loop restatements of TF-1 op index arithmetic, for tiny inputs only
(TEST INFRASTRUCTURE ONLY).  They pin the torch-based oracle in oracle/tf_ops.py and
oracle/geometry.py: two independent codings of the same formula must agree.
"""
import numpy as np


def same_pad(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return out, tot // 2


def conv2d_same(x, w, s):
    """y[n,o,p,co] = sum x[n, o*s-pt+i, p*s-pl+j, ci] * w[i,j,ci,co] (zero outside)."""
    N, H, W, C = x.shape
    kh, kw, _, K = w.shape
    OH, pt = same_pad(H, kh, s)
    OW, pl = same_pad(W, kw, s)
    y = np.zeros((N, OH, OW, K))
    for n in range(N):
        for o in range(OH):
            for p in range(OW):
                for i in range(kh):
                    for j in range(kw):
                        yy, xx = o * s - pt + i, p * s - pl + j
                        if 0 <= yy < H and 0 <= xx < W:
                            y[n, o, p] += x[n, yy, xx] @ w[i, j]
    return y


def conv2d_transpose_same(x, w, s=2):
    """Scatter form of Conv2DBackpropInput: out[n, s*i+a-pt, s*j+b-pl, co] += x[n,i,j,ci] w[a,b,co,ci]."""
    N, h, wd, C = x.shape
    kh, kw, K, _ = w.shape
    H, W = s * h, s * wd
    _, pt = same_pad(H, kh, s)
    _, pl = same_pad(W, kw, s)
    y = np.zeros((N, H, W, K))
    for n in range(N):
        for i in range(h):
            for j in range(wd):
                for a in range(kh):
                    for b in range(kw):
                        o, p = s * i + a - pt, s * j + b - pl
                        if 0 <= o < H and 0 <= p < W:
                            y[n, o, p] += w[a, b] @ x[n, i, j]
    return y


def resize_nearest(x, oh, ow):
    N, H, W, C = x.shape
    sy, sx = np.float32(H) / np.float32(oh), np.float32(W) / np.float32(ow)
    y = np.zeros((N, oh, ow, C))
    for i in range(oh):
        for j in range(ow):
            y[:, i, j] = x[:, min(int(np.floor(np.float32(i) * sy)), H - 1),
                           min(int(np.floor(np.float32(j) * sx)), W - 1)]
    return y


def resize_bilinear(x, oh, ow):
    N, H, W, C = x.shape
    sy, sx = np.float32(H) / np.float32(oh), np.float32(W) / np.float32(ow)
    y = np.zeros((N, oh, ow, C))
    for i in range(oh):
        fy = np.float32(i) * sy
        y0 = int(np.floor(fy)); y1 = min(y0 + 1, H - 1); ly = fy - y0
        for j in range(ow):
            fx = np.float32(j) * sx
            x0 = int(np.floor(fx)); x1 = min(x0 + 1, W - 1); lx = fx - x0
            top = x[:, y0, x0] * (1 - lx) + x[:, y0, x1] * lx
            bot = x[:, y1, x0] * (1 - lx) + x[:, y1, x1] * lx
            y[:, i, j] = top + (bot - top) * ly
    return y


def bilinear_sample(img, coords):
    """utils_lr.py:309-366 per pixel: unclamped floor for the weights, clamp for the indices,
    a clamped tap's weight is zero."""
    B, Hs, Ws, C = img.shape
    _, Ht, Wt, _ = coords.shape
    out = np.zeros((B, Ht, Wt, C))
    wm = np.zeros((B, Ht, Wt, 1))
    for b in range(B):
        for i in range(Ht):
            for j in range(Wt):
                x, y = coords[b, i, j]
                x0, y0 = np.floor(x), np.floor(y)
                acc = np.zeros(C); ws = 0.0
                for xx, wx in ((x0, x0 + 1 - x), (x0 + 1, x - x0)):
                    for yy, wy in ((y0, y0 + 1 - y), (y0 + 1, y - y0)):
                        xs, ys = min(max(xx, 0), Ws - 1), min(max(yy, 0), Hs - 1)
                        wgt = (wx if xs == xx else 0.0) * (wy if ys == yy else 0.0)
                        acc += wgt * img[b, int(ys), int(xs)]
                        ws += wgt
                out[b, i, j] = acc
                wm[b, i, j, 0] = ws
    return out, wm
