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
contribution of the step (`uses` backward calls per chunk) is launched at once, so the exchange of one network
overlaps the other network's chain (and, with several buckets, the backward conv of its own early layers).
`join()` / `finish()` launch any bucket never reported before the Adam that reads it.

Over RCCL the collectives are direct `ncclAllReduce` calls on communicators of our own (rccl.py: one per parameter
chunk, i.e. per network, created in chunk order on every rank) -- ProcessGroupNCCL, its Work objects, events and
watchdog thread are not in the data path.  The replicas' SUM stays in chunk.grad; Adam applies 1/world as it loads
the gradient (`grad_scale`, read by train.Adam at every update; no scale pass).  (ReduceOp.AVG would fold the scale
into RCCL, but RCCL runs AVG as a pre-multiplied sum with an extra kernel per call: at world 1 a oneRankReduce copy
pass, 52 calls x 219 us per config-4 step, profiles/r05/bench_ab_exchange_sum.md.)  Two modes:
  * "segments" (the default): a launch point joins the reporting program's filter-gradient branch into its stream;
    under capture it closes the current graph segment, and replay runs segment, the bucket's all-reduce issued by the
    host on THAT stream, next segment ...  No collective is inside a graph, no extra stream exists (round 6: a
    dedicated comm stream shared one of the GPU_MAX_HW_QUEUES = 4 FIFO hardware queues with a compute chain and cost
    28 % at world 1, profiles/r06/bench_r06c_xseg_*), and each network's Adam follows its own exchange inline on its
    stream.  Every collective is issued by one host thread in program order, each communicator from one stream: the
    same sequence on every rank whatever the GPU timing (tests/test_ddp.py `order`);
  * "graph" (opt-in, rounds 5-6): the all-reduces are CAPTURED.  A launch point first joins the chunk's filter-gradient
    branch into the current (capture) stream (pre_launch), then forks the chunk's comm stream off that stream alone --
    every fork of the capture is ONE level deep (round 6: round 5 made the comm branch also wait on the
    filter-gradient branch, a fork of a fork, the shape DESIGN.md §5 records as crashing hipStreamEndCapture) -- and
    the bucket's all-reduce becomes a graph node on that branch; `join(chunk)` at the end of the program's backward
    joins it back, so no graph is cut.  With the net overlap two graphs replay concurrently on two streams:
    Trainer refuses graph mode with it at world > 1.
  Bucket size: measured on one GPU (config 4, world-1 RCCL, bench.py --exchange on), every mid-backward launch point
  costs a join of the filter-gradient branch (and, in segments mode, a graph cut); DESIGN.md §6 derives the default,
  one bucket per network (256 MB), from a world-8 model.
Over gloo (CPU tensors, or GPU tensors in tests/test_gpu_ddp_world2.py) the launch goes through torch.distributed
(on a comm stream for GPU tensors) and leaves the mean.

On CPU (gloo, device 'cpu') the same bookkeeping runs synchronously; tests/test_ddp.py drives it with
world_size 2.
"""
import torch

from . import _lib


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

    chunks: ParamChunks updated by the step; uses: {id(chunk): backward calls per step} (default 1).

    Over RCCL (GPU tensors, nccl backend) every chunk all-reduces on a direct RCCL communicator of its own
    (rccl.pooled_comm: created in chunk order on every rank, so chunk i's communicator is the same everywhere) and the
    replicas' SUM stays in chunk.grad: `grad_scale` = 1/world is what the optimizer applies (train.Adam reads it at
    every update).  `inline` (segments mode over RCCL): the all-reduce is issued on the stream of the network that
    reports the bucket, so its Adam may follow in the same stream (Trainer._inline_adam).  Over gloo the collectives
    run through torch.distributed and leave the mean (grad_scale 1)."""

    def __init__(self, chunks, world, bucket_mb=32.0, uses=None, group=None, pre_launch=None, side_streams=None,
                 mode=None, pre_fork=None):
        self.world, self.group = world, group
        # pre_launch(chunk): joins the streams that write the chunk's gradients beside the current stream (its
        # program's filter-gradient branch, NetProgram.join_wgrad) into it.  Called before every graph-mode fork (so
        # the comm branch forks from the current stream alone), before every RCCL launch point of segments mode
        # (the all-reduce follows on that stream) and, under capture, before a segment ends (a graph segment can
        # only end with its forked branches joined).  Over gloo on GPU tensors (eager) the compute stream never
        # waits: side_streams(chunk) lists those streams and the comm stream waits on an event at each one's tail.
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
        self.capturing = None       # set by Trainer.capture: callable(buckets) closing a graph segment
        self.log = []               # launch order (names), for tests
        nccl = self._rccl(group)
        self.rccl = nccl
        self.mode = mode or "segments"
        if self.mode not in ("graph", "segments") or (self.mode == "graph" and not nccl):
            raise ValueError(f"exchange mode {self.mode!r}: 'graph' needs RCCL (nccl backend), else 'segments'")
        self.captured = self.mode != "segments"
        self.inline = nccl and not self.captured
        # what the optimizer multiplies the exchanged gradient by: over RCCL the replicas' SUM stays in chunk.grad (no
        # scale pass), over gloo the launch leaves the mean
        self.grad_scale = 1.0 / world if nccl else 1.0
        # gloo on GPU tensors: one dedicated comm stream (a HIP stream of its own, never one of torch's pooled streams,
        # which a capture stream may alias)
        self.comm = self._new_stream() if (self.gpu and not nccl) else None
        # over RCCL: per chunk a direct communicator (and in graph mode a comm stream) of its own
        # pre_fork(chunk): issue whatever the chunk's program still holds back for its side streams (the deferred
        # filter-gradient calls) before a launch point records events on them
        self.pre_fork = pre_fork
        self.comm_of, self.group_of = {}, {}
        if nccl:
            for i, c in enumerate(self.chunks):
                self.group_of[id(c)] = self._chunk_comm(i, group)
                if self.captured:
                    self.comm_of[id(c)] = self._new_stream()
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
    def _chunk_comm(i, group):
        from .rccl import pooled_comm
        return pooled_comm("exchange", i, group)

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
    def _all_reduce(view, comm):
        comm.all_reduce_sum(view)      # on the current stream

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
        elif self.inline:
            if self.pre_launch is not None and chunk is not None:
                self.pre_launch(chunk)   # the all-reduce follows the chunk's filter gradients on this stream
            self.launch(buckets)
        else:
            self.launch(buckets, self.side_streams(chunk) if (self.side_streams and chunk is not None) else ())

    # ---- the exchange
    def launch(self, buckets, streams=()):
        """Segments mode.  Over RCCL: all-reduce (SUM) `buckets` on the CURRENT stream, each on its chunk's
        communicator (at replay: the stream of the piece whose segment just ended, which joined its filter-gradient
        branch before the cut).  Over gloo: on the comm stream after everything issued so far on the current stream
        and on `streams` (events: neither the current stream nor the side streams wait), then the 1/world scale."""
        import torch.distributed as dist
        self.log.extend(list(b.names) for b in buckets)
        if self.rccl:
            for b in buckets:
                self._all_reduce(b.view(), self.group_of[id(b.chunk)])
            return
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
        """End of a program's backward (its Adam may follow).  Graph mode: launch the chunk's buckets never reported
        on its branch, then order the current stream after its comm stream.  Inline segments mode: the chunk's
        unreported buckets become a launch point of their own (under capture a segment cut), so they are reduced
        before the Adam that follows on this stream."""
        rest = [b for b in self.buckets if b.chunk is chunk and not b.launched]
        if self.captured:
            if rest:
                for b in rest:
                    b.launched = True
                self.launch_forked(rest, chunk)
            if id(chunk) in self.forked:
                self._wait(self._current(), self.comm_of[id(chunk)])
                self.forked.discard(id(chunk))
        elif self.inline and rest:
            self._ready(rest, chunk)

    def leftovers(self):
        return [b for b in self.buckets if not b.launched]

    def finish(self, streams=()):
        """Launch what was never reported (after `streams` too), then order the compute stream after the comm
        stream (gloo on GPU tensors)."""
        if self.captured:
            for c in self.chunks:
                self.join(c)
            return
        rest = self.leftovers()
        if rest:
            for b in rest:
                b.launched = True
            self.launch(rest, streams)
        if self.comm is not None:
            torch.cuda.current_stream().wait_stream(self.comm)

    def __call__(self):
        """Non-overlapped fallback used when backward ran without hooks: everything after backward."""
        self.finish()
