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

Under hipGraph capture (Trainer.capture) a launch point instead closes the current graph segment;
replay runs segment, launches its buckets eagerly, next segment ... so RCCL stays outside graphs.

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

    chunks: ParamChunks updated by the step; uses: {id(chunk): backward calls per step} (default 1)."""

    def __init__(self, chunks, world, bucket_mb=32.0, uses=None, group=None, pre_launch=None, side_streams=None):
        self.world, self.group = world, group
        # pre_launch(chunk): called before a bucket launch point UNDER CAPTURE -- joins the streams that write the
        # chunk's gradients beside the capture stream (its program's filter-gradient branch, NetProgram.join_wgrad),
        # since a graph segment can only end with its forked branches joined.  Eagerly the compute stream never
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
        # a dedicated HIP stream (never one of torch's pooled streams, which a capture stream may alias)
        self.comm = _lib.dedicated_stream() if self.gpu else None
        self.capturing = None       # set by Trainer.capture: callable(buckets) closing a graph segment
        self.log = []               # launch order (names), for tests
        self.begin_step()

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
        if self.capturing is not None:
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

    def leftovers(self):
        return [b for b in self.buckets if not b.launched]

    def finish(self, streams=()):
        """Launch what was never reported (after `streams` too), then order the compute stream after the comm
        stream."""
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
