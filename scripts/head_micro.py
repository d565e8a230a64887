"""Head-kernel micro-benchmark (diagnostic): us per tde_head_fwd / tde_head_bwd call at the reference nets'
high-resolution head shapes.   python scripts/head_micro.py   (TDE_HEAD_TILE=0/1, TDE_HEAD_RW=0/1 select the path)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_depth_estimation_amd import _lib  # noqa: E402

L = _lib
lib = L.load()
st = L.stream_ptr()
SHAPES = [  # name, N, H, W, C, K, k
    ("disp1_b16", 16, 192, 256, 16, 1, 3), ("disp2_b16", 16, 96, 128, 32, 1, 3), ("disp3_b16", 16, 48, 64, 64, 1, 3),
    ("disp1", 8, 192, 256, 16, 1, 3), ("disp2", 8, 96, 128, 32, 1, 3), ("mask1", 8, 192, 256, 16, 2, 7),
    ("mask2", 8, 96, 128, 32, 2, 5), ("flow1", 32, 192, 256, 16, 2, 3), ("c5disp1", 2, 480, 640, 16, 1, 3),
    ("mask1_b16", 16, 192, 256, 16, 2, 7), ("mask2_b16", 16, 96, 128, 32, 2, 5)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


for name, N, H, W, C, K, k in SHAPES:
    d = L.ConvDesc()
    d.N, d.H, d.W, d.C, d.OH, d.OW, d.K, d.KH, d.KW = N, H, W, C, H, W, K, k, k
    d.stride, d.pad_top, d.pad_left, d.w_cin = 1, (k - 1) // 2, (k - 1) // 2, C
    d.x_cstride, d.x_coff, d.y_cstride, d.y_coff = C, 0, K, 0
    x = torch.randn(N, H, W, C, device="cuda")
    w = torch.randn(k, k, C, K, device="cuda") * 0.1
    b = torch.zeros(K, device="cuda")
    y = torch.empty(N, H, W, K, device="cuda")
    dy = torch.randn(N, H, W, K, device="cuda")
    dx = torch.empty_like(x)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    ws = torch.empty(lib.tde_head_workspace_size(ctypes.byref(d)) // 4 + 64, device="cuda")
    f = lambda: L.check(lib.tde_head_fwd(ctypes.byref(d), L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(y), 1, 4.0, 0.0, st))
    g = lambda: L.check(lib.tde_head_bwd(ctypes.byref(d), L.ptr(x), L.ptr(w), L.ptr(y), L.ptr(dy), L.ptr(dx), 0,
                                         L.ptr(dw), L.ptr(db), 0, 1, 4.0, 0.0, L.ptr(ws), ws.numel() * 4, st))
    gd = lambda: L.check(lib.tde_head_bwd(ctypes.byref(d), L.ptr(x), L.ptr(w), L.ptr(y), L.ptr(dy), L.ptr(dx), 0,
                                          None, None, 0, 1, 4.0, 0.0, L.ptr(ws), ws.numel() * 4, st))
    tf, tb, td = timeit(f), timeit(g), timeit(gd)
    print(f"{name:8s} fwd {tf:7.1f} us  bwd(dx+dw) {tb:7.1f} us  bwd(dx only) {td:7.1f} us", flush=True)
