"""Diagnostic (not collected by pytest): error statistics of one conv's FWD and WGRAD per conv math mode
against a float64 reference -- rms and mean signed error (bias) relative to rms(ref).

    python tests/diag_conv_err.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import tf_ops as T  # noqa: E402
from test_gpu_kernels import conv_desc, ws_for  # noqa: E402

from tf_depth_estimation_amd import _lib as L  # noqa: E402


def stats(g, r):
    e = g.double().cpu() - r
    s = r.pow(2).mean().sqrt()
    return f"rms {(e.pow(2).mean().sqrt() / s).item():.2e} bias {(e.mean() / s).item():+.2e} " \
           f"max {(e.abs().max() / r.abs().max()).item():.2e}"


def main():
    lib = L.load()
    st = L.stream_ptr()
    for (N, H, W, C, K, k, scale) in [(8, 24, 32, 256, 256, 3, 1.0), (8, 48, 64, 64, 64, 3, 1.0),
                                      (8, 24, 32, 256, 256, 3, 1e-3)]:
        g = torch.Generator().manual_seed(0)
        x = torch.rand(N, H, W, C, generator=g, dtype=torch.float64) * scale   # post-ReLU-like (>= 0)
        w = (torch.rand(k, k, C, K, generator=g, dtype=torch.float64) - 0.5) * 0.1
        dy = torch.randn(N, H, W, K, generator=g, dtype=torch.float64)
        OH, pt, _ = T.same_pad(H, k, 1)
        OW, pl, _ = T.same_pad(W, k, 1)
        xr = x.clone().requires_grad_(True)
        wr = w.clone().requires_grad_(True)
        yr = T.conv2d_same(xr, wr, 1)
        yr.backward(dy)
        d = conv_desc(L, N=N, H=H, W=W, C=C, OH=OH, OW=OW, K=K, KH=k, KW=k, stride=1, pad_top=pt, pad_left=pl,
                      w_cin=C, x_cstride=C, x_coff=0, y_cstride=K, y_coff=0)
        ws = ws_for(L, d)
        gx, gw, gdy = x.float().cuda(), w.float().cuda(), dy.float().cuda()
        # reference on the fp32-rounded inputs
        xr32 = x.float().double().requires_grad_(True)
        wr32 = w.float().double().requires_grad_(True)
        y32 = T.conv2d_same(xr32, wr32, 1)
        y32.backward(dy.float().double())
        for m in (0, 2, 3):
            L.check(lib.tde_set_conv_math(m))
            gy = torch.empty(N, OH, OW, K, device="cuda")
            L.check(lib.tde_conv2d_fwd(ctypes.byref(d), L.ptr(gx), L.ptr(gw), L.ptr(gy), 0, L.ptr(ws),
                                       ws.numel() * 4, st))
            gdw = torch.empty_like(gw)
            L.check(lib.tde_conv2d_bwd_filter(ctypes.byref(d), L.ptr(gx), L.ptr(gdy), L.ptr(gdw), 0, L.ptr(ws),
                                              ws.numel() * 4, st))
            gdx = torch.empty_like(gx)
            L.check(lib.tde_conv2d_bwd_data(ctypes.byref(d), L.ptr(gdy), L.ptr(gw), L.ptr(gdx), 0, L.ptr(ws),
                                            ws.numel() * 4, st))
            torch.cuda.synchronize()
            print(f"{N}x{H}x{W}x{C}->{K} k{k} s{scale:g} math {m}: fwd {stats(gy, y32.detach())} | "
                  f"dgrad {stats(gdx, xr32.grad)} | wgrad {stats(gdw, wr32.grad)}", flush=True)
        # fp32 CPU (torch) for scale
        y_cpu = T.conv2d_same(x.float(), w.float(), 1)
        print(f"   cpu fp32 fwd {stats(y_cpu, y32.detach())}", flush=True)
    L.check(lib.tde_set_conv_math(3))


if __name__ == "__main__":
    main()
