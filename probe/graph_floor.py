"""Per-kernel cost of back-to-back tiny kernels in a torch-captured hipGraph (diagnostic)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_depth_estimation_amd import _lib  # noqa: E402

lib = _lib.load()
K = 200
x = torch.zeros(1 << 20, device="cuda")
st = lambda: _lib.stream_ptr()


def timed(fn, label):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    print(f"{label:40s} {a.elapsed_time(b) * 1e3 / (10 * K):6.2f} us/kernel", flush=True)


timed(lambda: [lib.tde_scale(16, _lib.ptr(x), 0.5, st()) for _ in range(K)], "tde_scale n=16")
timed(lambda: [lib.tde_scale(1 << 20, _lib.ptr(x), 0.5, st()) for _ in range(K)], "tde_scale n=1M")
timed(lambda: [lib.tde_zero_bytes(64, _lib.ptr(x), st()) for _ in range(K)], "tde_zero_bytes 64B")
timed(lambda: [x[:16].mul_(0.5) for _ in range(K)], "torch mul_ n=16")
