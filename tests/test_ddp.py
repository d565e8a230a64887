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
    """The default exchange is "segments" (round 6) and leaves the MEAN in chunk.grad (grad_scale 1 for Adam);
    "graph" mode (the bucket all-reduces captured as graph nodes) needs the nccl backend and is refused otherwise.
    Graph mode all-reduces with SUM and hands Adam grad_scale = 1 / world (tde_adam_update's grad_scale; the RCCL
    side is checked by tests/test_gpu_ddp.py)."""
    _, chunk = _chunk()
    gs = ddp.GradSync([chunk], 4, bucket_mb=1.0)
    assert gs.mode == "segments" and not gs.captured and gs.grad_scale == 1.0
    with pytest.raises(ValueError):
        ddp.GradSync([chunk], 4, bucket_mb=1.0, mode="graph")


class _Stream:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return self.name


class _TopologySync(ddp.GradSync):
    """GradSync in graph mode with its stream / collective primitives recorded instead of run: the fork/join topology
    a captured step would build, on CPU."""
    cur = None
    ops = None

    def _rccl(self, group):
        return True

    def _new_stream(self):
        return _Stream(f"comm{len(self.ops) if self.ops is not None else 0}_{id(self) % 997}")

    @staticmethod
    def _chunk_comm(i, group):
        return f"{group or 'world'}/comm{i}"

    def _current(self):
        return _TopologySync.cur

    def _on(self, stream):
        import contextlib

        @contextlib.contextmanager
        def ctx():
            prev, _TopologySync.cur = _TopologySync.cur, stream
            try:
                yield
            finally:
                _TopologySync.cur = prev
        return ctx()

    def _wait(self, waiter, waitee):
        _TopologySync.ops.append(("wait", waiter, waitee))

    def _all_reduce(self, view, group):
        _TopologySync.ops.append(("allreduce", _TopologySync.cur, group))


@pytest.mark.parametrize("mb", [1.0, 256.0])
def test_graph_mode_forks_one_level_deep(mb):
    """the graph-mode exchange's fork/join topology under a (recorded) capture.  The capture
    stream `cap` has one side branch, the program's filter-gradient stream `wgrad` (forked by the program, joined by
    pre_launch = Trainer._join_chunk_wgrad).  Every comm branch must fork from the capture stream ALONE, after the
    filter-gradient branch was joined into it: no stream forks from a branch, and the comm stream never waits on the
    filter-gradient stream.  Every comm branch is joined back before the step ends, its all-reduces run on it."""
    import ddp_worker
    spec, chunk = _chunk()
    cap, wgrad = _Stream("cap"), _Stream("wgrad")
    _TopologySync.ops, _TopologySync.cur = [], cap

    def join_wgrad(c):
        _TopologySync.ops.append(("wait", _TopologySync.cur, wgrad))

    def wgrad_fork():
        _TopologySync.ops.append(("wait", wgrad, cap))
    gs = _TopologySync([chunk], 2, bucket_mb=mb, mode="graph", pre_launch=join_wgrad,
                       side_streams=lambda c: (wgrad,), pre_fork=lambda c: None)
    assert gs.captured and gs.grad_scale == 0.5
    comm = gs.comm_of[id(chunk)]
    gs.begin_step()
    hook = gs.hook(chunk)
    for names in ddp_worker.schedule(spec):
        wgrad_fork()                      # the program forks its filter-gradient branch once per layer
        hook(names)
    join_wgrad(chunk)                     # the backward's own final join
    gs.join(chunk)
    ops = _TopologySync.ops
    # branches: a stream is a branch of `cap` once it waited on cap; a fork from a branch would be a wait whose
    # waitee is neither the capture stream nor the waiter's own parent joining back
    for kind, a, b in ops:
        if kind != "wait":
            continue
        if a is comm:
            assert b is cap, f"comm branch waits on {b!r}: a fork of a fork"
        if b is comm:
            assert a is cap, "comm branch joined into a side branch"
    waits_comm = [i for i, (k, a, b) in enumerate(ops) if k == "wait" and a is comm]
    assert waits_comm, "no bucket was forked"
    for i in waits_comm:                  # the filter-gradient branch was joined right before each fork
        assert ops[i - 1] == ("wait", cap, wgrad), ops[i - 1:i + 1]
    reduces = [(a, g) for k, a, g in ops if k == "allreduce"]
    assert len(reduces) == len(gs.buckets) and all(a is comm and g == "world/comm0" for a, g in reduces)
    assert ops[-1] == ("wait", cap, comm), "the comm branch is not joined back at the end"
    assert all(b.launched for b in gs.buckets)


@pytest.mark.parametrize("mode", ["graph", "segments"])
def test_every_chunk_reduces_on_a_communicator_of_its_own(mode):
    """one communicator under several chunks' streams would see their collectives in an order no rank
    controls.  Over RCCL every chunk gets a direct communicator of its own (rccl.pooled_comm by chunk index), with the
    default group and with an explicit one; segments mode over RCCL issues inline (no comm stream) and leaves the SUM
    for Adam's 1/world."""
    _, c1 = _chunk()
    _, c2 = _chunk()
    _TopologySync.ops = []
    for group in (None, "explicit"):
        gs = _TopologySync([c1, c2], 2, bucket_mb=1.0, mode=mode, group=group)
        assert gs.group_of[id(c1)] != gs.group_of[id(c2)]
        assert gs.grad_scale == 0.5 and gs.comm is None
        assert gs.inline == (mode == "segments")


def test_segments_inline_launch_order():
    """Segments mode over RCCL, eagerly: at each launch point the chunk's filter-gradient branch is joined into the
    current stream (pre_launch) and the bucket is all-reduced on that same stream, on the chunk's communicator."""
    import ddp_worker
    spec, chunk = _chunk()
    cap, wgrad = _Stream("cap"), _Stream("wgrad")
    _TopologySync.ops, _TopologySync.cur = [], cap
    gs = _TopologySync([chunk], 2, bucket_mb=4.0, mode="segments",
                       pre_launch=lambda c: _TopologySync.ops.append(("wait", _TopologySync.cur, wgrad)))
    gs.begin_step()
    hook = gs.hook(chunk)
    for names in ddp_worker.schedule(spec):
        hook(names)
    gs.join(chunk)
    gs.finish()
    ops = _TopologySync.ops
    red = [i for i, o in enumerate(ops) if o[0] == "allreduce"]
    assert len(red) == len(gs.buckets) and all(ops[i][1] is cap for i in red)
    for i in red:     # each launch point: join, then its bucket(s) on the same stream
        j = i
        while ops[j - 1][0] == "allreduce":
            j -= 1
        assert ops[j - 1] == ("wait", cap, wgrad), ops[j - 1:i + 1]


def test_adam_reads_grad_scale_from_the_exchange():
    """every Adam behind a trainer's optimizer (MultiAdam's sub-optimizers included) reads the exchange's
    gradient convention at update time: 1/world while graph mode leaves the SUM in chunk.grad, 1 when unlinked."""
    from tf_depth_estimation_amd import train
    _, c1 = _chunk()
    _, c2 = _chunk()
    opt = train.MultiAdam([c1, c2])
    assert all(o.grad_scale == 1.0 for o in opt.opts)
    _TopologySync.ops = []
    gs = _TopologySync([c1, c2], 4, bucket_mb=1.0, mode="graph")
    train.link_grad_scale(opt, gs)
    assert all(o.grad_scale == 0.25 for o in opt.opts)
    gs.grad_scale = 0.125                 # read at call time, not copied at link time
    assert all(o.grad_scale == 0.125 for o in opt.opts)
    train.link_grad_scale(opt, None)
    assert all(o.grad_scale == 1.0 for o in opt.opts)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("case", ["mean", "uses2", "two_programs", "oracle_step", "syncbn", "order"])
def test_gloo_world2(case):
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "ddp_worker.py"),
           case]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert f"ddp_worker {case} ok (world 2)" in r.stdout
