"""Micro-benchmark of the implicit-GEMM conv kernels on fixed shapes (diagnostic).

    python scripts/conv_micro.py [--math fp32|bf16x3|both] [--reps 20]
For each shape and mode (fwd / dgrad / wgrad) prints the mean HIP-event time and TFLOP/s."""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tf_depth_estimation_amd import _lib  # noqa: E402
from tf_depth_estimation_amd.program import same_pad  # noqa: E402

SHAPES = [
    # name, N, H, W, C, K, k, s
    ("gemm1x1_big", 8, 64, 64, 512, 512, 1, 1),
    ("big3x3", 32, 48, 64, 256, 256, 3, 1),
    ("cnv1b", 8, 96, 128, 32, 32, 7, 1),
    ("cnv2b", 8, 48, 64, 64, 64, 5, 1),
    ("icnv4", 8, 24, 32, 256, 128, 3, 1),
    ("icnv5", 8, 12, 16, 512, 256, 3, 1),
    ("icnv6", 8, 6, 8, 1024, 512, 3, 1),
    ("cnv4b", 8, 12, 16, 256, 256, 3, 1),
    ("icnv1", 8, 192, 256, 20, 16, 3, 1),
    ("icnv2", 8, 96, 128, 68, 32, 3, 1),
    ("icnv3", 8, 48, 64, 132, 64, 3, 1),
    ("cnv7", 8, 3, 4, 512, 512, 3, 2),
    ("cnv7b", 8, 2, 2, 512, 512, 3, 1),
    ("icnv7", 8, 2, 2, 1024, 512, 3, 1),
    ("cnv6b", 8, 3, 4, 512, 512, 3, 1),
    # deconvs as their virtual convs (x = deconv output, y = deconv input): "dgrad" = the deconv forward,
    # "fwd" = its data gradient
    ("upcnv1", 8, 192, 256, 16, 32, 3, 2),
    ("upcnv2", 8, 96, 128, 32, 64, 3, 2),
    ("upcnv3", 8, 48, 64, 64, 128, 3, 2),
    ("upcnv4", 8, 24, 32, 128, 256, 3, 2),
    ("upcnv5", 8, 12, 16, 256, 512, 3, 2),
    ("upcnv6", 8, 6, 8, 512, 512, 3, 2),
    # the same at config 4's twin batch (16 = the two calls of one network)
    ("upcnv1_b16", 16, 192, 256, 16, 32, 3, 2),
    ("upcnv2_b16", 16, 96, 128, 32, 64, 3, 2),
    ("upcnv3_b16", 16, 48, 64, 64, 128, 3, 2),
    # config 4's stride-2 layers at the twin batch (pixel-shuffle forms: deconv forward / conv dgrad, filter gradient)
    ("cnv1p_b16", 16, 192, 256, 8, 32, 7, 2),
    ("cnv1c4_b16", 16, 192, 256, 4, 32, 7, 2),
    ("cnv2_b16", 16, 96, 128, 32, 64, 5, 2),
    ("cnv3_b16", 16, 48, 64, 64, 128, 3, 2),
    ("cnv4_b16", 16, 24, 32, 128, 256, 3, 2),
    ("expup1_b16", 16, 192, 256, 16, 32, 7, 2),
    # stride-1 64-output-channel layers at the twin batch (halo-tiled filter gradient candidates)
    ("cnv2b_b16", 16, 48, 64, 64, 64, 5, 1),
    ("cnv1b_b16", 16, 96, 128, 32, 32, 7, 1),
    ("icnv1_b16", 16, 192, 256, 20, 16, 3, 1),
    ("icnv3_b16", 16, 48, 64, 132, 64, 3, 1),
    ("icnv2_b16", 16, 96, 128, 68, 32, 3, 1),
    ("cnv3b_b16", 16, 24, 32, 128, 128, 3, 1),
    ("cnv4b_b16", 16, 12, 16, 256, 256, 3, 1),
    ("icnv4_b16", 16, 24, 32, 260, 128, 3, 1),
    ("icnv5_b16", 16, 12, 16, 512, 256, 3, 1),
]


def run(lib, name, N, H, W, C, K, k, s, reps, modes=("fwd", "dgrad", "wgrad"), acc=0):
    OH, pt = same_pad(H, k, s)
    OW, pl = same_pad(W, k, s)
    d = _lib.ConvDesc(N=N, H=H, W=W, C=C, OH=OH, OW=OW, K=K, KH=k, KW=k, stride=s, pad_top=pt, pad_left=pl,
                      w_cin=C, x_cstride=C, x_coff=0, y_cstride=K, y_coff=0)
    x = torch.randn(N, H, W, C, device="cuda")
    w = torch.randn(k, k, C, K, device="cuda") * 0.1
    y = torch.randn(N, OH, OW, K, device="cuda")
    dx, dw = torch.zeros_like(x), torch.zeros_like(w)
    wsz = max(lib.tde_conv2d_workspace_size(ctypes.byref(d), o) for o in range(3))
    ws = torch.zeros(wsz // 4 + 16, device="cuda")
    st = _lib.stream_ptr()
    flops = 2.0 * N * OH * OW * K * k * k * C
    calls = {
        "fwd": lambda: lib.tde_conv2d_fwd(ctypes.byref(d), _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), acc, _lib.ptr(ws),
                                          ws.numel() * 4, st),
        "dgrad": lambda: lib.tde_conv2d_bwd_data(ctypes.byref(d), _lib.ptr(y), _lib.ptr(w), _lib.ptr(dx), acc,
                                                 _lib.ptr(ws), ws.numel() * 4, st),
        "wgrad": lambda: lib.tde_conv2d_bwd_filter(ctypes.byref(d), _lib.ptr(x), _lib.ptr(y), _lib.ptr(dw), acc,
                                                   _lib.ptr(ws), ws.numel() * 4, st),
    }
    out = []
    for mode, fn in calls.items():
        if mode not in modes:
            continue
        for _ in range(3):
            _lib.check(fn(), mode)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        out.append((mode, ms, flops / ms / 1e9))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--math", default="both")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--modes", default="fwd,dgrad,wgrad")
    ap.add_argument("--accumulate", type=int, default=0)
    a = ap.parse_args()
    lib = _lib.load()
    modes = [_lib.CONV_MATH[m] for m in _lib.CONV_MATH] if a.math in ("both", "all") else \
        [_lib.CONV_MATH[m] for m in a.math.split(",")]
    for m in modes:
        _lib.check(lib.tde_set_conv_math(m))
        print(f"== math {[k for k, v in _lib.CONV_MATH.items() if v == m][0]}")
        for sh in SHAPES:
            if a.shapes and sh[0] not in a.shapes.split(","):
                continue
            res = run(lib, *sh, a.reps, a.modes.split(","), a.accumulate)
            print(f"{sh[0]:12s} " + "  ".join(f"{mode} {ms * 1e3:7.1f}us {tf:6.1f}TF" for mode, ms, tf in res),
                  flush=True)


if __name__ == "__main__":
    main()
