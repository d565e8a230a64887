"""Data-parallel host logic on CPU: gradient buckets and the overlapped exchange.

In-process tests check the bucket partition against the real disp_net parameter layout; the
world_size-2 cases run tests/ddp_worker.py under torch.distributed.run with the gloo backend (the same
launcher bench.py uses for N > 1, with RCCL in place of gloo on the GPU box)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tf_depth_estimation_amd import ddp  # noqa: E402


def _chunk():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ddp_worker
    return ddp_worker.build()


@pytest.mark.parametrize("mb", [0.25, 1.0, 4.0, 1024.0])
def test_buckets_partition_flat_gradient(mb):
    spec, chunk = _chunk()
    bs = ddp.make_buckets(chunk, int(mb * 2 ** 20))
    # launch order = from the end of the buffer; contiguous, disjoint, covering [0, numel)
    assert bs[0].hi == chunk.numel and bs[-1].lo == 0
    for a, b in zip(bs, bs[1:]):
        assert a.lo == b.hi
    seen = [n for b in bs for n in b.names]
    assert sorted(seen) == sorted(chunk.names()) and len(seen) == len(set(seen))
    cap = int(mb * 2 ** 20)
    for b in bs:
        assert b.nbytes <= cap or len(b.names) == 1, (b.nbytes, b.names)
        for n in b.names:
            o = chunk.offsets[n]
            assert b.lo <= o and o + chunk.grad_view(n).numel() <= b.hi
    if mb >= 1024:
        assert len(bs) == 1


def test_bucket_launches_follow_backward_schedule():
    """With the real reverse-op schedule each bucket fires exactly once, at the very op that reports
    the last of its parameters (never before, never later), and the first fires well before the end."""
    import ddp_worker
    spec, chunk = _chunk()
    gs = ddp.GradSync([chunk], 1, bucket_mb=1.0)
    fired, cur = {}, [None]

    def fake_launch(buckets, streams=()):
        for b in buckets:
            assert id(b) not in fired
            fired[id(b)] = cur[0]
    gs.launch = fake_launch
    gs.begin_step()
    hook = gs.hook(chunk)
    sched = ddp_worker.schedule(spec)
    reported = {}
    for i, names in enumerate(sched):
        for n in names:
            reported[n] = i
        cur[0] = i
        hook(names)
    cur[0] = len(sched)
    gs.finish()
    assert len(fired) == len(gs.buckets)
    for b in gs.buckets:
        assert fired[id(b)] == max(reported[n] for n in b.names), b.names
    assert min(fired.values()) < len(sched) // 2


def test_exchange_mode_and_grad_scale():
    """Without RCCL the exchange runs in "segments" mode and leaves the MEAN in chunk.grad (grad_scale 1 for Adam);
    "graph" mode (the bucket all-reduces captured as graph nodes) needs the nccl backend and is refused otherwise.
    Graph mode all-reduces with SUM and hands Adam grad_scale = 1 / world (tde_adam_update's grad_scale; the RCCL
    side is checked by tests/test_gpu_ddp.py)."""
    _, chunk = _chunk()
    gs = ddp.GradSync([chunk], 4, bucket_mb=1.0)
    assert gs.mode == "segments" and not gs.captured and gs.grad_scale == 1.0
    with pytest.raises(ValueError):
        ddp.GradSync([chunk], 4, bucket_mb=1.0, mode="graph")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("case", ["mean", "uses2", "two_programs", "oracle_step", "syncbn"])
def test_gloo_world2(case):
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "ddp_worker.py"),
           case]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert f"ddp_worker {case} ok (world 2)" in r.stdout
