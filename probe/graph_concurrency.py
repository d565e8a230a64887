"""Diagnostic (round 3): do captured graphs replayed on two streams run concurrently on this stack?
Each chain is a run of small elementwise kernels (latency-bound, a few CUs each), so two chains side by side
take ~max(A, B) when they overlap and ~A + B when they are serialized.  Cases: two graphs (one pool, one
capture stream), two graphs on their own capture streams and pools, one graph beside an eager chain, and one
graph holding both chains as forked branches.
    python probe/graph_concurrency.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tf_depth_estimation_amd import _lib  # noqa: E402

N = 300


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


def report(name, ta, tb, tab):
    print(f"[graph_concurrency] {name}: A {ta:.3f} ms, B {tb:.3f} ms, A||B {tab:.3f} ms -> "
          f"{'CONCURRENT' if tab < 0.75 * (ta + tb) else 'serialized'} (max {max(ta, tb):.3f}, sum {ta + tb:.3f})",
          flush=True)


def main():
    xa, xb = torch.randn(256, 256, device="cuda"), torch.randn(256, 256, device="cuda")
    w = torch.randn(256, 256, device="cuda") * 0.05
    chain(xa, w, 2)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    s1, s2 = _lib.dedicated_stream(), _lib.dedicated_stream()

    def pair(fa, fb):
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

    # 0. two streams each spinning one 1-thread kernel (torch.cuda._sleep): hardware queue concurrency alone
    spin = 2_000_000
    sl = lambda: torch.cuda._sleep(spin)  # noqa: E731
    report("eager spin kernels", timed(sl), timed(sl), timed(pair(sl, sl)))
    gs1, gs2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    cap0 = _lib.dedicated_stream()
    with torch.cuda.graph(gs1, stream=cap0):
        for _ in range(4):
            torch.cuda._sleep(spin // 4)
    with torch.cuda.graph(gs2, stream=cap0):
        for _ in range(4):
            torch.cuda._sleep(spin // 4)
    report("graph spin kernels", timed(gs1.replay), timed(gs2.replay), timed(pair(gs1.replay, gs2.replay)))

    # 1. two graphs, one capture stream, one pool
    cap = _lib.dedicated_stream()
    pool = torch.cuda.graph_pool_handle()
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=cap, pool=pool):
        chain(xa, w)
    with torch.cuda.graph(gb, stream=cap, pool=pool):
        chain(xb, w)
    ta, tb = timed(ga.replay), timed(gb.replay)
    torch.cuda.synchronize()
    t = time.perf_counter()
    ga.replay()
    th = (time.perf_counter() - t) * 1e3
    torch.cuda.synchronize()
    print(f"[graph_concurrency] host time of one replay call ({N} kernels): {th:.3f} ms", flush=True)
    report("two graphs, shared pool", ta, tb, timed(pair(ga.replay, gb.replay)))

    # 2. two graphs, own capture streams and pools
    ca, cb = _lib.dedicated_stream(), _lib.dedicated_stream()
    ga2, gb2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga2, stream=ca):
        chain(xa, w)
    with torch.cuda.graph(gb2, stream=cb):
        chain(xb, w)
    report("two graphs, own pools", timed(ga2.replay), timed(gb2.replay), timed(pair(ga2.replay, gb2.replay)))

    # 3. a graph beside a host-light eager stream (a few long kernels)
    big = torch.randn(64, 1024, 1024, device="cuda")

    def eager_long():
        for _ in range(4):
            torch.tanh(big, out=big)
    report("graph || eager", ta, timed(eager_long), timed(pair(ga.replay, eager_long)))

    # 4. one graph, both chains as forked branches
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=cap, pool=pool):
        c = torch.cuda.current_stream()
        s1.wait_stream(c)
        s2.wait_stream(c)
        with torch.cuda.stream(s1):
            chain(xa, w)
        with torch.cuda.stream(s2):
            chain(xb, w)
        c.wait_stream(s1)
        c.wait_stream(s2)
    report("one graph, two branches", ta, tb, timed(g1.replay))
    print("[graph_concurrency] env DEBUG_CLR_GRAPH_PACKET_CAPTURE=" +
          os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "(unset)"), flush=True)


if __name__ == "__main__":
    main()
