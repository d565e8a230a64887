"""Diagnostic (round 3): chains of short kernels on two streams serialize on this stack (probe/graph_concurrency.py):
each kernel's grid takes the whole chip, so the other stream's kernels wait.  Do two streams with DISJOINT CU masks
(hipExtStreamCreateWithCUMask) run such chains side by side?  Two mask layouts (the first / second half of the CU
bits, even / odd bits), eager and as graphs.
    python probe/cu_mask.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

N = 300
_hip = ctypes.CDLL("libamdhip64.so")
_keep = []


def masked_stream(bits):
    """A non-blocking stream limited to the CUs whose bits are set (list of CU indices)."""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for b in bits:
        m[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = _hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), m)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed {rc}")
    _keep.append(s)
    return torch.cuda.ExternalStream(s.value)


def chain(x, w, n=N):
    for _ in range(n):
        x = torch.tanh(x * w + 0.1)
    return x


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    xa, xb = torch.randn(256, 256, device="cuda"), torch.randn(256, 256, device="cuda")
    w = torch.randn(256, 256, device="cuda") * 0.05
    big = torch.randn(64, 1024, 1024, device="cuda")
    chain(xa, w, 2)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    print(f"[cu_mask] {ncu} CUs", flush=True)
    layouts = {"halves": (list(range(ncu // 2)), list(range(ncu // 2, ncu))),
               "even_odd": (list(range(0, ncu, 2)), list(range(1, ncu, 2))),
               "full": (list(range(ncu)), list(range(ncu)))}
    for name, (ma, mb) in layouts.items():
        s1, s2 = masked_stream(ma), masked_stream(mb)

        def on(s, fn):
            def run():
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    fn()
                cur.wait_stream(s)
            return run

        def both(fa, fb):
            def run():
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                with torch.cuda.stream(s1):
                    fa()
                with torch.cuda.stream(s2):
                    fb()
                cur.wait_stream(s1)
                cur.wait_stream(s2)
            return run

        ca, cb = (lambda: chain(xa, w)), (lambda: chain(xb, w))
        bigk = lambda: torch.tanh(big, out=big)  # noqa: E731
        ta, tb = timed(on(s1, ca)), timed(on(s2, cb))
        tab = timed(both(ca, cb))
        tbig = timed(on(s1, bigk))
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga, stream=s1):
            chain(xa, w)
        with torch.cuda.graph(gb, stream=s2):
            chain(xb, w)
        tga, tgb = timed(on(s1, ga.replay)), timed(on(s2, gb.replay))
        tgab = timed(both(ga.replay, gb.replay))
        print(f"[cu_mask] {name}: eager chain A {ta:.3f} B {tb:.3f} A||B {tab:.3f} ms; graph chain A {tga:.3f} "
              f"B {tgb:.3f} A||B {tgab:.3f} ms; 268 MB tanh on stream A {tbig:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
