"""Data-parallel gradient exchange over the batch.

The reference is single-device (no tower / replica code), so this is new: one process
per GPU, each holding a batch shard, all parameters replicated, and after backward the mean of the
per-rank gradients.  The loss terms are batch means, so the mean of per-rank gradients is the
gradient of the global-batch loss up to BatchNorm, whose statistics stay per rank (local BN, the
SURVEY.md §8e default).

Layout: the gradients of one ParamChunk live in ONE flat fp32 buffer whose order follows the forward
op order, so backward finishes them roughly from the end of the buffer toward its start.  Buckets
are contiguous slices cut from the end at parameter boundaries (<= bucket_bytes each, a larger
parameter gets a bucket of its own).  `NetProgram.backward` reports each op's parameters as soon
as their gradient is written (`on_grads`); a bucket whose parameters have all received their last
contribution of the step (`uses` backward calls per chunk) is launched at once:
    event on the compute stream -> comm stream waits -> all_reduce(SUM) -> scale 1/world
so the exchange of late layers overlaps the backward conv of early ones.  `finish()` launches any
bucket never reported and makes the compute stream wait for the comm stream before Adam.

Under hipGraph capture there are two modes:
  * mode "segments" (the default; gloo and RCCL): a launch point closes the current graph segment (the program's
    filter-gradient branch joined first) and replay runs segment, its buckets eagerly, next segment ... so the
    collectives stay OUTSIDE the graphs.  Every all-reduce of a step is issued by the host thread, in replay order,
    on ONE comm stream and ONE communicator: the issue order is the program order on every rank, whatever the GPU
    timing (tests/test_ddp.py `order` case), and ProcessGroupNCCL's watchdog only ever polls events recorded
    eagerly.  Round 6 made this the default everywhere: the captured mode below
    aborted once in the driver's GPU suite (GPUTEST_r05, SIGABRT inside Trainer.capture) and no world > 1 run of it
    exists;
  * mode "graph" (opt-in, RCCL only, rounds 5-6): the all-reduces are CAPTURED.  A launch point first joins the
    chunk's filter-gradient branch into the current (capture) stream (pre_launch), then forks the chunk's comm stream
    off that stream alone -- every fork of the capture is ONE level deep (round 6: round 5 made the comm branch also
    wait on the filter-gradient branch, a fork of a fork, the shape DESIGN.md §5 records as crashing
    hipStreamEndCapture) -- and the bucket's all-reduce (ReduceOp.SUM) becomes a graph node on that branch;
    `join(chunk)` at the end of the program's backward joins it back, so no graph is cut.  Each chunk all-reduces on
    a communicator of its own (created in chunk order on every rank).  With the net overlap two graphs replay
    concurrently on two streams, so two communicators would run in an order no rank controls: Trainer refuses graph
    mode with the net overlap at world > 1, and an explicit `group` shared by several chunks is refused here.
    Bucket size: measured on one GPU (config 4, world-1 RCCL group, bench.py --exchange on), every comm-branch fork
    in the middle of a backward stalls the other network's chain (its wait packets sit in FIFO hardware queues shared
    with it, GPU_MAX_HW_QUEUES = 4): 32 / 64 / 128 MB buckets 782 / 720 / 897 pairs/s, one bucket per
    network (256 MB) 1049-1055, against 1089-1093 without the exchange -- hence Trainer.enable_ddp's 256 MB default
    (DESIGN.md §6 derives the same default from a world-8 model).
    The 1/world of the mean is NOT a pass of its own: chunk.grad holds the replicas' SUM after the exchange and Adam
    applies `grad_scale` (= 1/world) as it reads the gradient (train.Adam reads it from this object at every update).
    ReduceOp.AVG would fold the scale into RCCL instead, but RCCL runs AVG as a pre-multiplied sum with an extra kernel
    per call -- at world 1 a oneRankReduce copy pass, 52 calls x 219 us per config-4 step, measured 1048-1051 pairs/s
    against 1083-1087 with SUM (profiles/r05/bench_ab_exchange_sum.md).

On CPU (gloo, device 'cpu') the same bookkeeping runs synchronously; tests/test_ddp.py drives it with
world_size 2.
"""
import torch

from . import _lib

_GROUPS = {}


def pooled_group(purpose, idx):
    """The idx-th RCCL communicator of `purpose` ("exchange", "syncbn") over the default process group, created on
    first use and reused by every later trainer of this process (all ranks ask in the same order, so the i-th group
    of a purpose is the same communicator everywhere).  One new group per trainer would pile up communicators -- and
    their device buffers and proxy threads -- in a process that builds many trainers (the GPU tests).  Entries hold
    the default group they were made under, so a re-initialised default group gets fresh ones."""
    import torch.distributed as dist
    world = dist.distributed_c10d._get_default_group()
    key = (id(world), purpose, idx)
    hit = _GROUPS.get(key)
    if hit is None:
        hit = _GROUPS[key] = (world, dist.new_group(backend="nccl"))
    return hit[1]


class Bucket:
    __slots__ = ("chunk", "lo", "hi", "names", "launched", "opt")

    def __init__(self, chunk, lo, hi, names):
        self.chunk, self.lo, self.hi, self.names = chunk, lo, hi, list(names)
        self.launched = False
        self.opt = None     # the chunk's optimizer when the bucket is an Adam-overlap slice (train.py)

    def view(self):
        return self.chunk.grad[self.lo:self.hi]

    @property
    def nbytes(self):
        return 4 * (self.hi - self.lo)


def make_buckets(chunk, bucket_bytes):
    """Contiguous slices of chunk.grad, cut at parameter boundaries from the END of the buffer.
    Returned in launch order (last parameters first).  Every element of the flat buffer, padding
    included, belongs to exactly one bucket."""
    cap = max(1, bucket_bytes // 4)
    params = sorted(chunk.offsets.items(), key=lambda kv: kv[1])
    ends = [off for _, off in params[1:]] + [chunk.numel]
    spans = [(name, off, end) for (name, off), end in zip(params, ends)]
    buckets, cur, cur_hi = [], [], None
    for name, lo, hi in reversed(spans):
        if cur and cur_hi - lo > cap:
            buckets.append(Bucket(chunk, cur[-1][1], cur_hi, [n for n, _ in cur]))
            cur, cur_hi = [], None
        if cur_hi is None:
            cur_hi = hi
        cur.append((name, lo))
    if cur:
        buckets.append(Bucket(chunk, cur[-1][1], cur_hi, [n for n, _ in cur]))
    if buckets and params:
        assert buckets[-1].lo == 0
    return buckets


class GradSync:
    """Bucketed, overlapped gradient mean over the default process group (RCCL on GPU, gloo on CPU).

    chunks: ParamChunks updated by the step; uses: {id(chunk): backward calls per step} (default 1)."""

    def __init__(self, chunks, world, bucket_mb=32.0, uses=None, group=None, pre_launch=None, side_streams=None,
                 mode=None, pre_fork=None):
        self.world, self.group = world, group
        # pre_launch(chunk): joins the streams that write the chunk's gradients beside the current stream (its
        # program's filter-gradient branch, NetProgram.join_wgrad) into it.  Called before every graph-mode fork (so
        # the comm branch forks from the current stream alone) and, in segments mode, before a launch point under
        # capture (a graph segment can only end with its forked branches joined).  Eagerly in segments mode the
        # compute stream never waits: side_streams(chunk) lists those streams and the comm stream waits on an event
        # at each one's tail.
        self.pre_launch = pre_launch
        self.side_streams = side_streams
        self.chunks = list(chunks)
        self.buckets = []
        self.by_param = {}
        for c in self.chunks:
            for b in make_buckets(c, int(bucket_mb * 2 ** 20)):
                self.buckets.append(b)
                for n in b.names:
                    self.by_param[(id(c), n)] = b
        self.uses = {id(c): (uses or {}).get(id(c), 1) for c in self.chunks}
        self.pending = {}
        self.device = self.chunks[0].grad.device if self.chunks else torch.device("cpu")
        self.gpu = self.device.type == "cuda"
        # a dedicated HIP stream (never one of torch's pooled streams, which a capture stream may alias)
        self.comm = self._new_stream() if self.gpu else None
        self.capturing = None       # set by Trainer.capture: callable(buckets) closing a graph segment
        self.log = []               # launch order (names), for tests
        nccl = self._rccl(group)
        self.mode = mode or "segments"
        if self.mode not in ("graph", "segments") or (self.mode == "graph" and not nccl):
            raise ValueError(f"exchange mode {self.mode!r}: 'graph' needs RCCL (nccl backend), else 'segments'")
        if self.mode == "graph" and group is not None and len(self.chunks) > 1:
            #  graph mode gives every chunk a comm branch of its own; one explicit communicator under
            # several branches would see their collectives in an order no rank controls
            raise ValueError("exchange mode 'graph' with an explicit group and several parameter chunks: one "
                             "communicator would serve concurrent graph branches; use mode 'segments'")
        self.captured = self.mode != "segments"
        # what the optimizer multiplies the exchanged gradient by: graph mode leaves the replicas' SUM in chunk.grad
        # (no scale pass on the comm branch), segments mode the mean
        self.grad_scale = 1.0 / world if self.captured else 1.0
        # graph mode: per chunk a comm stream and a communicator of its own (same creation order on every rank)
        # pre_fork(chunk): issue whatever the chunk's program still holds back for its side streams (the deferred
        # filter-gradient calls) before a launch point records events on them
        self.pre_fork = pre_fork
        self.comm_of, self.group_of = {}, {}
        if self.captured:
            for i, c in enumerate(self.chunks):
                self.comm_of[id(c)] = self._new_stream()
                self.group_of[id(c)] = self._chunk_group(i) if group is None else group
        self.forked = set()         # chunks whose comm stream has work not yet joined (graph mode)
        self.begin_step()

    # ---- stream / collective primitives (tests/test_ddp.py replays the graph-mode topology through a subclass that
    # records them instead of touching HIP or a process group)
    def _rccl(self, group):
        import torch.distributed as dist
        return self.gpu and dist.is_initialized() and dist.get_backend(group) == "nccl"

    @staticmethod
    def _new_stream():
        return _lib.dedicated_stream()

    @staticmethod
    def _chunk_group(i):
        return pooled_group("exchange", i)

    @staticmethod
    def _current():
        return torch.cuda.current_stream()

    @staticmethod
    def _on(stream):
        return torch.cuda.stream(stream)

    @staticmethod
    def _wait(waiter, waitee):
        _lib.wait_stream(waiter, waitee)

    @staticmethod
    def _all_reduce(view, group):
        import torch.distributed as dist
        dist.all_reduce(view, op=dist.ReduceOp.SUM, group=group)

    # ---- per-step bookkeeping
    def begin_step(self):
        self.count = {k: 0 for k in self.by_param}
        self.left = {id(b): len(b.names) for b in self.buckets}
        for b in self.buckets:
            b.launched = False
        self.log = []

    def hook(self, chunk):
        """Callback for NetProgram.backward(on_grads=...): names whose gradient was just written."""
        cid = id(chunk)

        def on_grads(names):
            ready = []
            for n in names:
                key = (cid, n)
                b = self.by_param.get(key)
                if b is None:
                    continue
                self.count[key] += 1
                if self.count[key] == self.uses[cid]:
                    self.left[id(b)] -= 1
                    if self.left[id(b)] == 0:
                        ready.append(b)
            if ready:
                self._ready(ready, chunk)
        return on_grads

    def _ready(self, buckets, chunk=None):
        for b in buckets:
            b.launched = True
        if self.captured:
            self.launch_forked(buckets, chunk)
        elif self.capturing is not None:
            if self.pre_launch is not None:
                self.pre_launch(chunk)
            self.capturing(buckets)      # graph segment boundary; launched at replay
        else:
            self.launch(buckets, self.side_streams(chunk) if (self.side_streams and chunk is not None) else ())

    # ---- the exchange
    def launch(self, buckets, streams=()):
        """All-reduce `buckets` on the comm stream after everything issued so far on the current stream and on
        `streams` (events: neither the current stream nor the side streams wait for anything)."""
        import torch.distributed as dist
        self.log.extend(list(b.names) for b in buckets)
        if not self.gpu:
            for b in buckets:
                v = b.view()
                dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
                v.mul_(1.0 / self.world)
            return
        ev = torch.cuda.Event()
        ev.record()
        self.comm.wait_event(ev)
        for sd in streams:
            e2 = torch.cuda.Event()
            e2.record(sd)
            self.comm.wait_event(e2)
        lib = _lib.load()
        with torch.cuda.stream(self.comm):
            st = _lib.stream_ptr()
            for b in buckets:
                v = b.view()
                dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
                _lib.check(lib.tde_scale(v.numel(), _lib.ptr(v), 1.0 / self.world, st), "grad scale")

    def launch_forked(self, buckets, chunk):
        """Graph mode: all-reduce (sum; Adam applies 1/world) `buckets` on the chunk's comm stream.  The chunk's
        filter-gradient branch is first joined into the current stream (pre_launch: its deferred calls issued, then
        the current stream waits on its tail), and the comm stream is forked from the current stream ALONE -- one
        level deep under capture, where the all-reduces become graph nodes of a branch that join(chunk) merges back;
        eagerly the same stream order."""
        self.log.extend(list(b.names) for b in buckets)
        if chunk is None:
            chunk = buckets[0].chunk
        if self.pre_launch is not None:
            self.pre_launch(chunk)
        elif self.pre_fork is not None:
            self.pre_fork(chunk)
        comm = self.comm_of[id(chunk)]
        self._wait(comm, self._current())
        with self._on(comm):
            for b in buckets:
                self._all_reduce(b.view(), self.group_of[id(chunk)])
        self.forked.add(id(chunk))

    def join(self, chunk):
        """Graph mode: launch the chunk's buckets never reported, then order the current stream after its comm stream
        (the end of the program's backward: its Adam may follow)."""
        if not self.captured:
            return
        rest = [b for b in self.buckets if b.chunk is chunk and not b.launched]
        if rest:
            for b in rest:
                b.launched = True
            self.launch_forked(rest, chunk)
        if id(chunk) in self.forked:
            self._wait(self._current(), self.comm_of[id(chunk)])
            self.forked.discard(id(chunk))

    def leftovers(self):
        return [b for b in self.buckets if not b.launched]

    def finish(self, streams=()):
        """Launch what was never reported (after `streams` too), then order the compute stream after the comm
        stream."""
        if self.captured:
            for c in self.chunks:
                self.join(c)
            return
        rest = self.leftovers()
        if rest:
            for b in rest:
                b.launched = True
            self.launch(rest, streams)
        if self.gpu:
            torch.cuda.current_stream().wait_stream(self.comm)

    def __call__(self):
        """Non-overlapped fallback used when backward ran without hooks: everything after backward."""
        self.finish()
