"""Training steps for the BASELINE configs, as static schedules of libtde.so calls.

A step is fwd + fused loss head (forward and its hand-derived gradient in one pass) + bwd + Adam,
all on one HIP stream over buffers allocated once, so `Trainer.capture()` can record the whole step
into a hipGraph (torch.cuda.CUDAGraph) and replay it with zero host work per step.

  DepthOnlyTrainer   config 2 -- train_depth_only.py:108-219 (disp_net, smooth + depth L1, Adam)
"""
import os
import warnings

import torch

from . import _api, _lib, _netlib, variables
from ._lib import ptr
from .program import IN_PLACE, NetRun

W_CONFIG2 = dict(smooth=1.0, depth=1.0)     # train_depth_only.py:33-37

# Thread-local capture: RCCL's watchdog thread polls the events of earlier collectives while a step is
# being recorded; under the default "global" mode that poll is an illegal call during capture and
# aborts the process (hipErrorStreamCaptureUnsupported).
CAPTURE_MODE = "thread_local"


def _halves(a, b):
    """True when dense tensors a and b are the two consecutive halves of one buffer (b starts where a ends)."""
    return (a.is_contiguous() and b.is_contiguous() and a.shape == b.shape and
            b.data_ptr() == a.data_ptr() + a.numel() * a.element_size())


def _end_segment(g):
    """capture_end() of one graph segment; None when nothing was recorded into it (a bucket launch point right
    at a piece boundary).  An empty segment is dropped instead of replayed: its buckets launch after the
    previous segment, which is where the stream's tail already is."""
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        g.capture_end()
    empty = False
    for w in caught:
        if "CUDA Graph is empty" in str(w.message):
            empty = True
        else:
            warnings.warn_explicit(w.message, w.category, w.filename, w.lineno)
    return None if empty else g


class Adam:
    """tf.train.AdamOptimizer(lr, beta1) over one ParamChunk (flat buffers)."""

    def __init__(self, chunk, lr=2e-4, beta1=0.9, beta2=0.999, eps=1e-8):
        self.chunk, self.lr, self.b1, self.b2, self.eps = chunk, lr, beta1, beta2, eps
        self.t = torch.zeros(1, device=chunk.flat.device, dtype=torch.float32)
        # the exchange whose gradient convention applies (link_grad_scale / Trainer.enable_ddp): graph mode leaves
        # the replicas' SUM in chunk.grad, segments mode the mean
        self.scale_src = None

    @property
    def grad_scale(self):
        """What the gradient is multiplied by as Adam reads it, looked up at every update: 1/world
        while a captured exchange (ddp.GradSync graph mode) leaves the replicas' SUM in chunk.grad, else 1."""
        return 1.0 if self.scale_src is None else float(self.scale_src.grad_scale)

    def step(self):
        self.begin()
        self.update(0, self.chunk.numel)

    def begin(self):
        """Advance the device step counter (TF's beta1_power / beta2_power)."""
        lib, st = _lib.load(), _lib.stream_ptr()
        _lib.check(lib.tde_adam_step_begin(ptr(self.t), st), "adam step")

    def update(self, lo, hi):
        """Adam on flat elements [lo, hi) (multiples of 4: parameters start 16-byte aligned)."""
        import ctypes
        lib, st = _lib.load(), _lib.stream_ptr()
        c = self.chunk

        def at(t):
            return ctypes.c_void_p(t.data_ptr() + 4 * lo)
        _lib.check(lib.tde_adam_update(hi - lo, at(c.flat), at(c.grad), at(c.adam_m), at(c.adam_v), ptr(self.t),
                                       self.lr, self.b1, self.b2, self.eps, self.grad_scale, st), "adam")


def optimizers(opt):
    """The Adam instances behind a trainer's optimizer (an Adam or a MultiAdam)."""
    return list(opt.opts) if hasattr(opt, "opts") else [opt]


def link_grad_scale(opt, sync):
    """Make every Adam behind `opt` read its gradient scale from `sync` (a ddp.GradSync, or None to unlink)."""
    for o in optimizers(opt):
        o.scale_src = sync


class AdamOverlap:
    """Single-GPU overlap of the optimizer with backward: the gradient buffers are cut into buckets
    (ddp.make_buckets: contiguous slices, last parameters first) and each bucket's Adam runs on a side
    stream as soon as backward has written its last contribution of the step, so the update of the
    decoder's and the deep encoder's large layers hides under the remaining backward convs.  Pure
    kernel work: under capture the side stream becomes a graph branch (fork at each bucket's event,
    one join before the step ends)."""

    def __init__(self, opts, bucket_mb=16.0, uses=None, pre_launch=None, streams=None):
        from .ddp import make_buckets
        self.opts = list(opts)
        self.pre_launch = pre_launch
        # streams: {id(chunk): stream} -- run a chunk's buckets on that stream (its program's filter-gradient
        # stream, which already holds the chunk's last weight gradients in order: no join with it needed)
        self.streams = dict(streams or {})
        self.buckets = []
        self.by_param = {}
        for o in self.opts:
            for b in make_buckets(o.chunk, int(bucket_mb * 2 ** 20)):
                b.opt = o
                self.buckets.append(b)
                for n in b.names:
                    self.by_param[(id(o.chunk), n)] = b
        self.uses = {id(o.chunk): (uses or {}).get(id(o.chunk), 1) for o in self.opts}
        self.side = _lib.dedicated_stream()

    def begin_step(self):
        self.count = {k: 0 for k in self.by_param}
        self.left = {id(b): len(b.names) for b in self.buckets}
        self.done = set()
        for o in self.opts:
            o.begin()

    def hook(self, chunk):
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
                self.launch(ready)
        return on_grads

    def launch(self, buckets):
        # the event orders each update after everything the compute stream has issued so far: the op that
        # reported the gradients, and the data-gradient GEMM that still READ these parameters
        ev = torch.cuda.Event()
        ev.record()
        on_side = [b for b in buckets if id(b.chunk) not in self.streams]
        if on_side:
            if self.pre_launch is not None:
                self.pre_launch()
                ev = torch.cuda.Event()
                ev.record()
            _lib.wait_event(self.side, ev)
            with torch.cuda.stream(self.side):
                for b in on_side:
                    b.opt.update(b.lo, b.hi)
                    self.done.add(id(b))
        for b in buckets:
            st = self.streams.get(id(b.chunk))
            if st is None:
                continue
            _lib.wait_event(st, ev)
            with torch.cuda.stream(st):
                b.opt.update(b.lo, b.hi)
            self.done.add(id(b))

    def finish(self):
        rest = [b for b in self.buckets if id(b) not in self.done]
        if rest:
            self.launch(rest)
        _lib.wait_stream(torch.cuda.current_stream(), self.side)
        for st in set(self.streams.values()):
            _lib.wait_stream(torch.cuda.current_stream(), st)


class DeferredAdam:
    """Single-GPU: the optimizer step of step k runs at the START of step k+1 on a side stream, overlapped
    with that step's forward, which waits (per parameter bucket, in forward order) only for the buckets of
    the layers it is about to run.  Each chunk's flat buffer is cut into two buckets in forward order: the
    first layers (`first_mb`, updated in a few microseconds) and the rest, which the forward needs only when
    it reaches the deeper layers -- the high-resolution encoder layers run meanwhile.  The sequence of
    updates and their arithmetic are those of Adam after backward (bit-identical parameters and moments once
    flush() has applied the last step's update); the backward of step k+1 overwrites the gradients only after
    its forward has waited for every bucket, i.e. after Adam read them."""

    def __init__(self, opts, first_mb=2.0):
        self.opts = list(opts)
        self.side = _lib.dedicated_stream()
        self.buckets = {}
        for o in self.opts:
            c = o.chunk
            cap = int(first_mb * 2 ** 20) // 4
            offs = sorted(c.offsets.values())
            cut = max([v for v in offs if v <= cap] or [0])
            cuts = [0] + ([cut] if 0 < cut < c.numel else []) + [c.numel]
            self.buckets[id(c)] = [[lo, hi, None] for lo, hi in zip(cuts[:-1], cuts[1:])]
        self.pending = False     # an update (of the last step's gradients) is owed
        self.active = False      # this step's forward must wait for the side stream's buckets
        self.waited = set()

    def launch(self):
        """Start of a step: the owed update on the side stream, one event per bucket."""
        self.active, self.waited = False, set()
        if not self.pending:
            return
        cur = torch.cuda.current_stream()
        _lib.wait_stream(self.side, cur)
        with torch.cuda.stream(self.side):
            for o in self.opts:
                o.begin()
                for b in self.buckets[id(o.chunk)]:
                    o.update(b[0], b[1])
                    b[2] = torch.cuda.Event()
                    b[2].record()
        self.active, self.pending = True, False

    def _needed(self, prog, i):
        span = prog.op_param_span(i)
        if span is None:
            return []
        return [b for b in self.buckets.get(id(prog.chunk), []) if b[0] < span[1] and span[0] < b[1]]

    def pre_op(self, prog, i):
        if not self.active:
            return
        for b in self._needed(prog, i):
            if id(b) not in self.waited:
                _lib.wait_event(torch.cuda.current_stream(), b[2])
                self.waited.add(id(b))

    def params_ready(self, prog, i):
        return not self.active or all(id(b) in self.waited for b in self._needed(prog, i))

    def end_forward(self):
        """After the forward: every bucket waited for (the join of the side branch under capture)."""
        if self.active:
            cur = torch.cuda.current_stream()
            for bs in self.buckets.values():
                for b in bs:
                    if id(b) not in self.waited:
                        _lib.wait_event(cur, b[2])
                        self.waited.add(id(b))
            _lib.wait_stream(cur, self.side)
            self.active = False


class AllReduceGrads:
    """Data-parallel gradient exchange: ONE RCCL all-reduce (sum) of the chunk's flat fp32 gradient
    buffer, then a scale by 1/world inside the next Adam launch's input (the loss terms are batch
    means, so the mean of per-rank gradients equals the gradient of the global-batch mean)."""

    def __init__(self, chunk, world):
        self.chunk, self.world = chunk, world

    def __call__(self):
        import torch.distributed as dist
        dist.all_reduce(self.chunk.grad, op=dist.ReduceOp.SUM)
        lib, st = _lib.load(), _lib.stream_ptr()
        g = self.chunk.grad
        _lib.check(lib.tde_scale(g.numel(), ptr(g), 1.0 / self.world, st), "grad scale")


class Trainer:
    """Common capture/replay machinery.  A step is phase_compute (fwd, loss, bwd -- the first backward call of a chunk overwrites its gradients),
    the optional gradient exchange, then phase_update (Adam).  Without an exchange the whole step is
    one hipGraph.  With a ddp.GradSync, backward reports finished parameters and each full bucket's
    RCCL all-reduce is launched on a side stream while backward continues; under capture, every
    launch point closes a graph segment, and replay interleaves segments with the bucket launches
    (RCCL itself is never captured), then one graph for Adam after the comm stream joins."""

    graphs = None
    segments = None          # [(graph, buckets launched after it)] when capturing with a GradSync
    seg_update = None        # the segmented capture's update graph (None when Adam runs inline)
    grad_sync = None
    BACKWARD_USES = 1        # backward calls per chunk per step (shared-variable nets call it twice)

    adam_ov = None
    dadam = None
    _graph_owes = False      # deferred Adam: the captured step begins with an owed update
    net_stream = None        # enable_net_overlap: the second program's calls on their own stream

    det_ws = None            # enable_deterministic: workspace of the deterministic warp-loss scatter

    def enable_deterministic(self, on=True):
        """Run-to-run bit-identical steps: the warp loss head's scatter-add into the other view's disparity
        gradient (utils_lr.py:330-366 gather -> UnsortedSegmentSum in the reference) and its loss / dL/dP block
        sums use the fixed-point / fixed-order mode of tde_warp_loss (det_ws) instead of float atomics.  Every
        other kernel of the step is already order-deterministic (fixed-order split-K / BN / head reductions).
        Call before capture()."""
        from . import losses as Ls
        self.det_ws = Ls.det_workspace(self.N, self.H, self.W) if on else None
        return self

    def enable_net_overlap(self, on=True):
        """Run the calls of one network program concurrently with those of the other on a second stream
        (config 4: `depth_net` on both pairs beside `disp_net` on both images, forward and backward; under capture
        each piece is its own graph on its stream).  The two programs share no buffer, parameter, gradient or
        moving statistic, and each program's calls keep their order, so the step is bit-identical to the serial
        one.  With the data-parallel exchange each program's bucket launch points cut its own piece's graphs
        (enable_ddp).  Not combinable with the Adam overlaps or host-side (gloo) SyncBN; RCCL SyncBN gives each
        program its own communicator (enable_sync_bn)."""
        if on and (self.adam_ov is not None or self.dadam is not None or
                   (getattr(self, "sync_bn", False) and not getattr(self, "sync_bn_capturable", False))):
            raise ValueError("net overlap is for the step without Adam overlap / deferred Adam / host-side SyncBN")
        if on:
            self._check_sync_bn_streams(net=True)
            self._check_exchange_streams(net=True)
        self.net_stream = _lib.owned_stream(self, "net") if on else None
        return self

    def _overlap_stream(self):
        """The second stream when the overlap applies to this call (not under the instrumented eager step,
        whose per-family HIP-event timer records on one stream)."""
        if self.net_stream is None or any(getattr(p, "timer", None) is not None and not getattr(p.timer, "graph", False)
                                          for p in self.programs()):
            return None
        return self.net_stream

    def enable_deferred_adam(self, first_mb=2.0):
        """Run each step's Adam at the start of the next step, overlapped with its forward (DeferredAdam).
        The parameters then lag the gradients by one update until flush()."""
        if self.grad_sync is not None or self.adam_ov is not None:
            raise ValueError("deferred Adam is for the single-GPU step without another Adam overlap")
        if self.net_stream is not None:
            # the overlapped capture has no _begin() piece: a deferred update would never be launched
            raise ValueError("deferred Adam and net overlap are exclusive")
        opts = self.opt.opts if hasattr(self.opt, "opts") else [self.opt]
        self.dadam = DeferredAdam(opts, first_mb)
        for o in opts:
            # checkpoint.Saver and the read-out methods apply an owed update first (the parameters lag by one)
            o.chunk.pending_flush = self.flush
        for p in self.programs():
            # the backward overwrites the gradients the update reads: it starts after every bucket is done
            p.pre_op, p.params_ready, p.pre_backward = self.dadam.pre_op, self.dadam.params_ready, self.dadam.end_forward
        return self.dadam

    def flush(self):
        """Apply the update a deferred-Adam step still owes (before reading or saving the parameters).  In graph
        mode the captured step begins with the owed update unconditionally, so after an eager flush the next
        step() runs eagerly once (no update owed at its start) and replays resume after it (step())."""
        if self.dadam is not None and self.dadam.pending:
            self.phase_update()
            self.dadam.pending = False

    def enable_adam_overlap(self, bucket_mb=16.0, on_wgrad_stream=False):
        """Run each gradient bucket's Adam on a side stream as soon as backward finalises it (single GPU;
        with a data-parallel exchange the update must wait for the all-reduce).  on_wgrad_stream: on each
        program's filter-gradient stream (enable_wgrad_overlap first), behind the filter gradients it holds,
        so the compute stream never waits for it until the end of the step."""
        if self.grad_sync is not None:
            raise ValueError("Adam overlap is for the single-GPU step (the exchange orders Adam after it)")
        if self.net_stream is not None:
            raise ValueError("Adam overlap and net overlap are exclusive")
        opts = self.opt.opts if hasattr(self.opt, "opts") else [self.opt]
        streams = {}
        if on_wgrad_stream:
            for p in self.programs():
                if p.wgrad_stream is None or isinstance(p.wgrad_stream, str):
                    raise ValueError("on_wgrad_stream needs enable_wgrad_overlap() (a side stream) first")
                if len(p.wgrad_streams) > 1:
                    raise ValueError("on_wgrad_stream needs ONE filter-gradient stream (TDE_WGRAD_STREAMS=1)")
                streams[id(p.chunk)] = p.wgrad_stream
        self.adam_ov = AdamOverlap(opts, bucket_mb, {id(c): self.BACKWARD_USES for c in self.chunks},
                                   pre_launch=self.join_wgrad, streams=streams)
        return self.adam_ov

    def enable_wgrad_overlap(self, on=True, serial=False, only=None):
        """Filter gradients on a side stream, off the backward chain (NetProgram.enable_wgrad_overlap;
        serial=True: the same split calls on the compute stream, the bit-exact reference of the overlap).
        only: a list of program attribute names ("single", "pair", "prog") to restrict it to (the others keep
        the fused data + filter gradient launch on their own stream); default: TDE_WGRAD_PROGS (comma list) or
        every program."""
        if only is None and os.environ.get("TDE_WGRAD_PROGS"):
            only = [x for x in os.environ["TDE_WGRAD_PROGS"].split(",") if x]
        for name in ("prog", "single", "pair"):
            p = getattr(self, name, None)
            if p is None:
                continue
            p.enable_wgrad_overlap(on and (only is None or name in only), serial)
        return self

    def _check_sync_bn_streams(self, net=False):
        """RCCL SyncBN across replicas issues its all-reduces from every stream that runs a BatchNorm.  Per-program
        communicators keep each communicator on one stream, but with GPU_MAX_HW_QUEUES = 4 the kernels of different
        communicators may share a hardware queue in a different order on different GPUs, which no world > 1 run has
        checked: refuse SyncBN over more than one replica combined with the net overlap, and an explicit
        shared group with any overlap or the gradient exchange."""
        if not getattr(self, "sync_bn", False):
            return
        world = max((getattr(p, "bn_world", 1) for p in self.programs()), default=1)
        net = net or self.net_stream is not None
        if world > 1 and net:
            raise ValueError("SyncBN over RCCL at world > 1 runs its collectives from one stream: no net overlap "
                             "with it")
        if getattr(self, "_sync_bn_group", None) is not None and (net or self.grad_sync is not None):
            raise ValueError("SyncBN with an explicit process group shares one communicator over several streams: "
                             "no overlap or bucketed exchange with it")

    def _check_exchange_streams(self, net=False):
        """The captured exchange (GradSync graph mode) all-reduces each network's buckets on a communicator and graph
        branch of its own.  With the net overlap the two networks' graphs replay concurrently on two streams, so at
        world > 1 the two communicators' collectives would meet in an order no rank fixes: refused --
        segments mode (the default) issues every collective from the host, in program order, on one comm stream."""
        gs = self.grad_sync
        if gs is None or not getattr(gs, "captured", False) or gs.world <= 1:
            return
        if net or self.net_stream is not None:
            raise ValueError("the captured (graph-mode) gradient exchange at world > 1 with the net overlap would run "
                             "two communicators in an unfixed order: use exchange mode 'segments' (the default)")

    timeline = None           # program.StepTimeline (diagnostic, probe/step_timeline.py)

    def set_timeline(self, tl):
        self.timeline = tl
        for p in self.programs():
            p.timeline = tl

    def _tl(self, label):
        if self.timeline is not None:
            self.timeline.mark("trainer", "T", label)

    def join_wgrad(self):
        for p in self.programs():
            p.join_wgrad()

    def _begin(self):
        if self.adam_ov is not None:
            self.adam_ov.begin_step()
        if self.dadam is not None:
            self.dadam.launch()

    def _update(self):
        if self.adam_ov is not None:
            self.adam_ov.finish()
        elif self.dadam is not None:
            self.dadam.end_forward()      # (normally already joined: the forward waited for every bucket)
            self.dadam.pending = True
        else:
            self.phase_update()

    def _inline_adam(self):
        """Whether each program's Adam runs inside phase_compute right after its own backward (DepthThenCamTrainer)."""
        return False

    def _program_of(self, chunk):
        for p in self.programs():
            if p.chunk is chunk:
                return p
        return None

    def _join_chunk_wgrad(self, chunk):
        """Under capture: join the filter-gradient branch of the program owning `chunk` into the current (that
        program's) stream -- a graph segment must end with its forked branches joined.  Only that program's:
        the other program may be mid-capture on its own stream (net overlap)."""
        p = self._program_of(chunk)
        for q in ([p] if p is not None else self.programs()):
            q.join_wgrad()

    def _chunk_side_streams(self, chunk):
        """Eagerly: the streams besides the current one that write `chunk`'s gradients (its program's
        filter-gradient streams); the comm stream waits on events at their tails, nobody else waits."""
        p = self._program_of(chunk)
        if p is None:
            return ()
        wg = () if p.wgrad_stream is None or isinstance(p.wgrad_stream, str) else tuple(p.wgrad_streams)
        return wg

    def _flush_chunk_wgrad(self, chunk):
        """Issue the deferred filter-gradient calls of the program owning `chunk` on its side stream (a captured
        exchange launch point then waits on that stream's tail)."""
        p = self._program_of(chunk)
        for q in ([p] if p is not None else self.programs()):
            if q.wgrad_stream is not None:
                q._flush_wgrad()

    def enable_ddp(self, world, bucket_mb=256.0, group=None, mode=None):
        """Bucketed gradient all-reduce overlapped with backward (ddp.GradSync).  mode "segments" (the default since
        round 6): graphs cut at every bucket launch point and every collective issued eagerly by the host between
        segment replays, in program order, on one comm stream; "graph" (opt-in, RCCL): the all-reduces are captured
        into the step's graphs on a per-network comm branch forked one level deep, joined at the end of that network's
        backward (its Adam then runs inline, as in the single-GPU step) -- refused with the net overlap at world > 1
        (_check_exchange_streams).  256 MB = one bucket per network at config 4 (the world-8 model)."""
        from .ddp import GradSync
        if self.adam_ov is not None:
            raise ValueError("Adam overlap and the data-parallel exchange are exclusive")
        uses = {id(c): self.BACKWARD_USES for c in self.chunks}
        self.grad_sync = GradSync(self.chunks, world, bucket_mb=bucket_mb, uses=uses, group=group,
                                  pre_launch=self._join_chunk_wgrad, side_streams=self._chunk_side_streams, mode=mode,
                                  pre_fork=self._flush_chunk_wgrad)
        link_grad_scale(self.opt, self.grad_sync)
        self._check_sync_bn_streams()
        self._check_exchange_streams()
        return self.grad_sync

    def enable_sync_bn(self, world, group=None):
        """SyncBN: every BatchNorm of every network normalises over the rows of all `world`
        replicas (one all-reduce of fp64 per-channel sums per BN layer and direction, all row groups of a twin
        run in one) -- the reference's semantics at the global batch.

        Over RCCL the sums all-reduce on direct RCCL communicators of their own (rccl.py; one per program, created
        in program order on every rank: each program's collectives are issued from its one stream in a fixed order,
        so the two networks of config 4 may run on two streams, and none of them shares a communicator with the
        gradient exchange) and the step can be captured: the all-reduces become nodes of the graph, with no
        ProcessGroupNCCL event or watchdog involved.  Over gloo (host collectives) the step runs eagerly."""
        import torch.distributed as dist
        nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"

        def make_sync(g):
            def sync(t):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=g)
            return sync

        def make_rccl_sync(comm):
            def sync(t):
                comm.all_reduce_sum(t)       # on the current stream
            return sync

        from .rccl import pooled_comm
        for pi, p in enumerate(self.programs()):
            sync = make_rccl_sync(pooled_comm("syncbn", pi, group)) if nccl else make_sync(group)
            p.bn_sync, p.bn_world = sync, world
        self.sync_bn = True
        self.sync_bn_capturable = nccl
        self._sync_bn_group = group
        self._check_sync_bn_streams()

    def programs(self):
        return [p for p in (getattr(self, "prog", None), getattr(self, "single", None), getattr(self, "pair", None))
                if p is not None]

    def hook(self, chunk):
        """on_grads callback for NetProgram.backward (None without an overlapped exchange)."""
        if self.adam_ov is not None:
            return self.adam_ov.hook(chunk)
        gs = self.grad_sync
        return gs.hook(chunk) if gs is not None and hasattr(gs, "hook") else None

    def step_eager(self):
        gs = self.grad_sync
        if gs is not None and hasattr(gs, "begin_step"):
            gs.begin_step()
        self._begin()
        self.phase_compute()
        if gs is not None:
            gs()
        self._update()

    def segment_cuts(self):
        """Graph cuts the segmented exchange made in the captured step (0 without it, or in graph mode)."""
        seq = getattr(self, "ov_seq", None)
        if seq is not None:
            return sum(max(0, len(segs) - 1) for _, segs in seq if segs is not None)
        return max(0, len(self.segments) - 1) if self.segments is not None else 0

    def release_graphs(self):
        """Drop the captured graphs (their memory pools go with them); step() runs eagerly until the next capture."""
        self.graphs = self.segments = self.seg_update = None
        if hasattr(self, "ov_seq"):
            self.ov_seq = None
        if hasattr(self, "ov_upd"):
            self.ov_upd = None

    def capture(self, warmup=2, **kw):
        """Warm up on a side stream (allocates every lazily created buffer), then record.  Every cross-stream wait
        made while recording keeps its event alive (_lib.capture_scope: the capture_end crash of round 2)."""
        with _lib.capture_scope():
            return self._capture(warmup, **kw)

    def _capture(self, warmup=2):
        if getattr(self, "sync_bn", False) and not getattr(self, "sync_bn_capturable", False):
            raise NotImplementedError("SyncBN over gloo all-reduces on the host inside forward/backward: run step() "
                                      "eagerly")
        if self.dadam is not None and not self.dadam.pending:
            # the captured step must begin with an owed update, or step() would never replay it: one
            # eager warm-up step makes one owed
            warmup = max(warmup, 1)
        s = _lib.owned_stream(self, "capture_warmup")
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_eager()
        torch.cuda.current_stream().wait_stream(s)
        gs = self.grad_sync
        if gs is None or getattr(gs, "captured", False):
            g = torch.cuda.CUDAGraph()
            # deferred Adam: whether the captured step begins with an owed update (it is recorded only if one
            # is owed at capture time); step() replays only when that matches the owed state
            self._graph_owes = self.dadam is not None and self.dadam.pending
            if gs is not None:
                gs.begin_step()
            with torch.cuda.graph(g, stream=_lib.owned_stream(self, "capture"), capture_error_mode=CAPTURE_MODE):
                self._begin()
                self.phase_compute()
                if gs is not None:
                    gs.finish()     # (graph mode: the all-reduces are nodes of this graph)
                self._update()
            self.graphs = [g]
            return self.graphs
        if not hasattr(gs, "begin_step"):       # plain exchange after backward
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=_lib.owned_stream(self, "capture"), capture_error_mode=CAPTURE_MODE):
                self.phase_compute()
            with torch.cuda.graph(g2, stream=_lib.owned_stream(self, "capture"), capture_error_mode=CAPTURE_MODE):
                self.phase_update()
            self.graphs = [g1, g2]
            return self.graphs
        # segmented capture: graph boundaries at bucket launch points
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        cs = _lib.owned_stream(self, "capture")
        segs = []
        state = {"g": torch.cuda.CUDAGraph()}

        def cut(buckets):
            segs.append((_end_segment(state["g"]), list(buckets)))
            state["g"] = torch.cuda.CUDAGraph()
            state["g"].capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)

        gs.begin_step()
        gs.capturing = cut
        try:
            with torch.cuda.stream(cs):
                state["g"].capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)
                self.phase_compute()
                segs.append((_end_segment(state["g"]), gs.leftovers()))
                upd = None
                if not self._inline_adam():
                    # (over RCCL a program's Adam follows its own exchange inside phase_compute: no update graph)
                    upd = torch.cuda.CUDAGraph()
                    upd.capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)
                    self.phase_update()
                    upd.capture_end()
        finally:
            gs.capturing = None
        torch.cuda.synchronize()
        self.segments = segs
        self.seg_update = upd
        self.graphs = [g for g, _ in segs if g is not None] + ([upd] if upd is not None else [])
        return self.graphs

    def step(self):
        if self.graphs is None:
            self.step_eager()
        elif self.segments is not None:
            gs = self.grad_sync
            gs.begin_step()
            for g, buckets in self.segments:
                if g is not None:
                    g.replay()
                if buckets:
                    for b in buckets:
                        b.launched = True
                    gs.launch(buckets)
            gs.finish()
            if self.seg_update is not None:
                self.seg_update.replay()
        elif len(self.graphs) == 1:
            if self.dadam is not None and self.dadam.pending != self._graph_owes:
                # an eager flush() (checkpoint save, read-out) already applied the update the graph would apply
                # first: one eager step (which owes nothing at its start), after which replays line up again
                self.step_eager()
                return
            self.graphs[0].replay()
            if self.dadam is not None:
                self.dadam.pending = True     # the replayed step's own update is owed
        else:
            self.graphs[0].replay()
            self.grad_sync()
            self.graphs[1].replay()


class DepthOnlyTrainer(Trainer):
    """Config 2: `train_depth_only.py` canonical interpretation:
    pred = nets_optflow_depth.disp_net(image_left) (:108); for s in 0..3:
      smooth += w_s/2^s * compute_smooth_loss(pred[s])                      (:167-168)
      depth  += mean|resize_area(label, s) - pred[s]| * w_d/2^s             (:170,183-184)
    total = depth + smooth (:219); Adam(lr, beta1) (:345-377)."""

    def __init__(self, batch, H=192, W=256, lr=2e-4, beta1=0.9, weights=W_CONFIG2, scope="model"):
        self.N, self.H, self.W, self.w = batch, H, W, weights
        with variables.variable_scope(scope):
            self.prog = _api.get_program("depth_net", _netlib.disp_net_spec, H, W, 3, decay=0.99, scale=4.0,
                                         offset=0.0)
        self.chunk = self.prog.chunk
        self.chunks = [self.chunk]
        self.run = NetRun(self.prog, batch)
        self.opt = Adam(self.chunk, lr, beta1)
        dev = "cuda"
        # the batch lives in the program's own input buffer (forward(run, IN_PLACE): no input copy), and the
        # loss head writes the output gradients straight into the program's gradient views (IN_PLACE)
        self.images = self.run.input_tensor()
        self.images.zero_()
        self.label = torch.ones(batch, H, W, 1, device=dev, dtype=torch.float32)
        outs = self.prog.spec.outputs
        self.d_out = [IN_PLACE] * len(outs)
        self.loss = torch.zeros(1, dtype=torch.float64, device=dev)
        self.parts = torch.zeros(2, dtype=torch.float64, device=dev)   # [depth, smooth]
        a = _lib.DepthLoss()
        a.N, a.H, a.W, a.nscales = batch, H, W, 4
        for s, v in enumerate(outs):
            a.pred[s] = self.run.vptr(v).value + 4 * v.coff   # 1-channel view of the net output
            a.pred_cs[s], a.pred_co[s] = v.buf.cs, 0
            a.grad[s] = self.run.grad_tensor(v).data_ptr()
            a.g_cs[s], a.g_co[s] = v.buf.cs, 0
            a.smooth_w[s] = self.w["smooth"] / 2 ** s        # train_depth_only.py:167-168
            a.l1_w[s] = self.w["depth"] / 2 ** s             # :183-184
        a.recip, a.nonfinite, a.grad_accumulate = 0, 0, 0
        a.label = self.label.data_ptr()
        a.loss_smooth = self.parts.data_ptr() + 8
        a.loss_l1 = self.parts.data_ptr()
        self.loss_args = a

    def set_batch(self, images, label):
        self.images.copy_(images)
        self.label.copy_(label)

    def phase_update(self):
        self.opt.step()

    def phase_compute(self):
        lib, st = _lib.load(), _lib.stream_ptr()
        _lib.check(lib.tde_zero_bytes(16, ptr(self.parts), st), "zero loss")
        outs = self.prog.forward(self.run, IN_PLACE, True)
        # the whole loss head (4 scales x (smooth + L1 to the area-downsampled label)) in one launch that
        # WRITES the output gradients (no zeroed gradient buffers)
        _lib.check(lib.tde_loss_depth_pyramid(ctypes_ref(self.loss_args), st), "depth loss head")
        # one backward call per step writes every parameter gradient: overwrite, no zeroed buffer
        self.prog.backward(self.run, self.d_out, on_grads=self.hook(self.prog.chunk), grad_accumulate=False)

    def total_loss(self):
        return float(self.parts.sum().item())

    def outputs(self):
        return [self.run.view_tensor(v) for v in self.prog.spec.outputs]


def ctypes_ref(x):
    import ctypes
    return ctypes.byref(x)


def ctypes_double_ptr(t, idx):
    import ctypes
    return ctypes.c_void_p(t.data_ptr() + 8 * idx)


class MultiAdam:
    def __init__(self, chunks, lr=2e-4, beta1=0.9):
        self.opts = [Adam(c, lr, beta1) for c in chunks]

    def step(self):
        for o in self.opts:
            o.step()


class MultiAllReduce:
    """One RCCL all-reduce per parameter chunk (flat, contiguous) + 1/world scale."""

    def __init__(self, chunks, world):
        self.parts = [AllReduceGrads(c, world) for c in chunks]

    def __call__(self):
        for p in self.parts:
            p()


def _scale_shapes(B, H, W, C, n=4):
    return [(B, H >> s, W >> s, C) for s in range(n)]


class DepthThenCamTrainer(Trainer):
    """Config 4: `train_depth_then_cam_lr.py` (canonical interpretation):
    single `disp_net` on each image (shared variables, separate BN batches, :123-136), 4-scale pair
    `depth_net` (nets_optflow_depth_pairtest) on concat(L,R) and concat(R,L) (:142-154), and per scale
    (:211-340): smoothness of 1/disp on the 4 maps, depth L1 with replace_nonfinite on the single left
    net, explainability-masked photometric warp + exp CE + left-right depth consistency in both
    directions, cam loss at s = 0; total (:355); Adam over both nets (:413-417).

    twin=True (default): each network's two calls run as ONE row-grouped call of batch 2B (NetRun groups=2):
    [left; right] images through disp_net, [concat(L,R); concat(R,L)] through depth_net -- every conv once over
    both sub-batches (the deep levels' GEMMs get twice the rows per launch, half the launches), every BatchNorm
    per sub-batch (the reference's separate BN batches), one backward per network summing both calls' parameter
    gradients.  twin=False: the four separate calls (the reference's literal schedule)."""

    SLOTS = dict(smooth=0, depth=1, photo=2, exp=3, consist=4, cam=5)

    def __init__(self, batch, H=192, W=256, lr=2e-4, beta1=0.9, weights=None, twin=True):
        from .losses import W_CONFIG4, Arena, new
        self.N, self.H, self.W = batch, H, W
        self.w = weights or W_CONFIG4
        self.twin = bool(twin)
        self.ov_net = "pair"   # the network on the second stream (net overlap); disp_net there measured 999 vs 1045
        self.BACKWARD_USES = 1 if self.twin else 2     # backward calls per chunk per step
        with variables.variable_scope("model_singledepth"):
            self.single = _api.get_program("depth_net", _netlib.disp_net_spec, H, W, 3, decay=0.99, scale=4.0,
                                           offset=0.0)
        with variables.variable_scope("model_pairdepth"):
            self.pair = _api.get_program("depth_cam_net", _netlib.depth_net_spec, H, W, 6, levels=4)
        self.chunks = [self.single.chunk, self.pair.chunk]
        self.opt = MultiAdam(self.chunks, lr, beta1)
        B = batch
        so, po = self.single.spec.outputs, self.pair.spec.outputs
        if self.twin:
            self.runs = {"s": NetRun(self.single, 2 * B, groups=2), "p": NetRun(self.pair, 2 * B, groups=2)}
            # images: [left; right] in one tensor, the single net's batched input; the pair net's input
            # [concat(L,R); concat(R,L)] (:146,152)
            self.img_lr = new((2 * B, H, W, 3))
            self.img = {"l": self.img_lr[:B], "r": self.img_lr[B:]}
            self.pair_in = new((2 * B, H, W, 6))
        else:
            self.runs = {k: NetRun(p, B) for k, p in (("sl", self.single), ("sr", self.single), ("pl", self.pair),
                                                       ("pr", self.pair))}
            self.img = {"l": new((B, H, W, 3)), "r": new((B, H, W, 3))}
            self.pair_in = {"lr": new((B, H, W, 6)), "rl": new((B, H, W, 6))}
        self.label = new((B, H, W, 1))
        self.K = new((B, 4, 3, 3))
        self.gt_cam = new((B, 6))
        if self.twin:
            # both images' area pyramids in one launch per scale (halves of [2B, H>>s, W>>s, 3] tensors)
            self.pyr_lr = [self.img_lr] + [new(s) for s in _scale_shapes(2 * B, H, W, 3)[1:]]
            self.pyr = {"l": [t[:B] for t in self.pyr_lr], "r": [t[B:] for t in self.pyr_lr]}
        else:
            self.pyr = {k: [self.img[k]] + [new(s) for s in _scale_shapes(B, H, W, 3)[1:]] for k in ("l", "r")}
        self.Ks = [new((B, 9)) for _ in range(4)]
        # the two directions' pose vectors (and gradients) as halves of one [2B, 6] tensor: with twin batching the
        # pose maps of the pair net's two calls are the halves of one output, so one spatial-mean launch serves both
        self.pose2, self.g_pose2 = new((2 * B, 6)), new((2 * B, 6))
        self.pose = {"lr": self.pose2[:B], "rl": self.pose2[B:]}
        self.g_pose = {"lr": self.g_pose2[:B], "rl": self.g_pose2[B:]}
        self.T = {"lr": new((B, 16)), "rl": new((B, 16))}
        self.P = {d: [new((B, 12)) for _ in range(4)] for d in ("lr", "rl")}
        self.Kinv = [new((B, 9)) for _ in range(4)]
        # everything the loss head accumulates into (loss parts, dL/dP, dL/dT, the runs' output gradients) lives
        # in one arena: one zeroing launch per step; the output gradients are the runs' own gradient buffers
        # (backward reads them in place)
        ar = Arena()
        ia = ar.new((8,), torch.float64)
        igp = {d: ar.new((4, B, 12), torch.float64) for d in ("lr", "rl")}
        igt = {d: ar.new((B, 16)) for d in ("lr", "rl")}
        nb = 2 * B if self.twin else B
        ido = {k: [ar.new((nb, v.H, v.W, v.C)) for v in (so if k[0] == "s" else po)] for k in self.runs}
        t = ar.finalize()
        self.arena = ar
        self.acc = t[ia]
        self.gP = {d: t[i] for d, i in igp.items()}
        self.gT = {d: t[i] for d, i in igt.items()}
        d_run = {k: [t[i] for i in idx] for k, idx in ido.items()}
        for k, run in self.runs.items():
            run.bind_output_grads(d_run[k])
        if self.twin:
            # the loss head addresses the four calls' outputs / output gradients as the halves of the batched runs
            self.d_run = d_run
            self.d_out = {}
            for k, half in (("sl", 0), ("sr", 1), ("pl", 0), ("pr", 1)):
                self.d_out[k] = [g[half * B:(half + 1) * B] for g in d_run[k[0]]]
        else:
            self.d_out = d_run

    def set_batch(self, img_l, img_r, label, K, gt_cam):
        """img_* [B,H,W,3] in [-0.5,0.5]; label = inverse depth [B,H,W,1] (NaN holes allowed);
        K [B,4,3,3] per-scale intrinsics (Demon_Data_loader.py:135-138); gt_cam [B,6] = (t, r)."""
        self.img["l"].copy_(img_l)
        self.img["r"].copy_(img_r)
        self.label.copy_(label)
        self.K.copy_(K)
        self.gt_cam.copy_(gt_cam)
        for s in range(4):
            self.Ks[s].copy_(self.K[:, s].reshape(-1, 9))

    def phase_update(self):
        if not self._inline_adam():
            self.opt.step()

    # phase_compute in pieces: "main" pieces on the compute stream, "ov" pieces (depth_net's calls) on the
    # second stream under enable_net_overlap.  Under capture each piece is its own graph (a whole program
    # forked onto a captured side branch made capture_end crash in a long-lived process -- ROCm 7 graph
    # instantiation, not reproducible alone), and replay interleaves them with stream waits.
    def _pieces(self):
        """The step as stream pieces: depth_net's chain (`ov_net` = "pair") on the second stream, issued before
        disp_net's on the compute stream.  disp_net's outputs enter only its own loss terms (smoothness of both maps,
        the depth L1 of the left; train_depth_then_cam_lr.py:211-355, oracle.losses.loss_depth_then_cam_lr), so each
        network's forward -> loss -> backward -> Adam is an independent chain: ONE join at the end of the step, and
        the depth_net-dependent loss runs beside disp_net's backward.  The second stream waits only for the inputs
        (concat + image area pyramids).  (Round 3's two-join schedule, TDE_C4_CHAINS=0, was deleted in round 5.)"""
        chain = {"pair": self._chain_pair, "single": self._chain_single}
        o = self.ov_net if self.ov_net in chain else "pair"
        m = "single" if o == "pair" else "pair"
        return [("main", self._p_inputs), ("ov", chain[o]), ("main", chain[m]), ("join", None)]

    def _chain_pair(self):
        self._chain_pair_a()
        self._chain_pair_b()

    def _chain_single(self):
        self._chain_single_a()
        self._chain_single_b()

    def _chain_pair_a(self):
        self._tl("pair chain start")
        self._p_fwd_pair()

    def _chain_pair_b(self):
        self._p_loss()
        self._tl("pair loss")
        self._p_bwd_pair()

    def _chain_single_a(self):
        self._tl("single chain start")
        self._p_fwd_single()

    def _chain_single_b(self):
        self._tl("single pyramids")
        self._p_bwd_single()

    def _p_inputs(self):
        self._tl("inputs start")
        self._p_concat()
        self._area_pyramids()
        self._tl("inputs")

    def _p_concat(self):
        lib, st = _lib.load(), _lib.stream_ptr()
        M = self.N * self.H * self.W
        self.arena.zero()
        # pair inputs: tf.concat([L, R], axis=3) and [R, L] (:146,152)
        if self.twin:
            # channels 0-2 of [concat(L,R); concat(R,L)] are [L; R] = img_lr: one copy for both halves
            _lib.check(lib.tde_copy_view(2 * M, 3, ptr(self.img_lr), 3, 0, ptr(self.pair_in), 6, 0, 0, st), "concat")
            _lib.check(lib.tde_copy_view(M, 3, ptr(self.img["r"]), 3, 0, ptr(self.pair_in[:self.N]), 6, 3, 0, st),
                       "concat")
            _lib.check(lib.tde_copy_view(M, 3, ptr(self.img["l"]), 3, 0, ptr(self.pair_in[self.N:]), 6, 3, 0, st),
                       "concat")
            return
        for key, (a, b) in (("lr", ("l", "r")), ("rl", ("r", "l"))):
            if self.twin:
                dst = self.pair_in[:self.N] if key == "lr" else self.pair_in[self.N:]
            else:
                dst = self.pair_in[key]
            _lib.check(lib.tde_copy_view(M, 3, ptr(self.img[a]), 3, 0, ptr(dst), 6, 0, 0, st), "concat")
            _lib.check(lib.tde_copy_view(M, 3, ptr(self.img[b]), 3, 0, ptr(dst), 6, 3, 0, st), "concat")

    def _halves(self, net, outs):
        """Twin run outputs -> the two calls' outputs: net "s" -> "sl" (left image) / "sr", "p" -> "pl" (pair L,R)
        / "pr" (pair R,L)."""
        B = self.N
        return {net + "l": [o[:B] for o in outs], net + "r": [o[B:] for o in outs]}

    def _p_fwd_pair(self):
        if self.twin:
            self._out.update(self._halves("p", self.pair.forward(self.runs["p"], self.pair_in)))
        else:
            self._out["pl"] = self.pair.forward(self.runs["pl"], self.pair_in["lr"])
            self._out["pr"] = self.pair.forward(self.runs["pr"], self.pair_in["rl"])

    def _p_fwd_single(self):
        if self.twin:
            self._out.update(self._halves("s", self.single.forward(self.runs["s"], self.img_lr)))
        else:
            self._out["sl"] = self.single.forward(self.runs["sl"], self.img["l"])
            self._out["sr"] = self.single.forward(self.runs["sr"], self.img["r"])
        from . import losses as Ls
        # the loss terms that need only this network's outputs and the inputs run here, on this network's stream:
        # disp_net's smoothness + depth-L1 pyramids in one launch; the rest of the loss needs depth_net's outputs
        # (_p_loss)
        Ls.pyramid_multi([self._pyramid_map(k) for k in ("sr", "sl")])

    def _area_pyramids(self):
        from . import losses as Ls
        for s in range(1, 4):
            if self.twin:
                Ls.area(self.img_lr, self.pyr_lr[s])
            else:
                Ls.area(self.img["l"], self.pyr["l"][s])
                Ls.area(self.img["r"], self.pyr["r"][s])

    def _pyramid_map(self, k):
        """Arguments of one map's smoothness of 1/disp at every scale (:216-225); on the single left net also the
        depth L1 to the area-downsampled label with replace_nonfinite (:227-232,241-243)."""
        w, S = self.w, self.SLOTS
        m = dict(preds=self._out[k][:4], grads=self.d_out[k][:4], acc=self.acc,
                 smooth_w=[w["smooth"] / 2 ** s for s in range(4)], slot_smooth=S["smooth"], recip=True)
        if k == "sl":
            m.update(label=self.label, l1_w=[w["depth"]] * 4, slot_l1=S["depth"], nonfinite=True)
        return m

    # each net runs twice (shared variables): the first backward call overwrites its gradients, the second
    # accumulates -- no zeroed gradient buffer needed.  Twin: one call per net overwrites them.
    def _bwd(self, k, prog, first):
        prog.backward(self.runs[k], [IN_PLACE] * len(self.runs[k].prog.spec.outputs), on_grads=self.hook(prog.chunk),
                      grad_accumulate=not first)

    def _inline_adam(self):
        """Plain step (no exchange, no Adam overlap / deferral): each network's Adam runs right after its own
        backward on that backward's stream -- depth_net's update overlaps disp_net's backward tail (and the
        other way round) instead of both updates waiting for the join.  The same update arithmetic."""
        gs = self.grad_sync
        return ((gs is None or getattr(gs, "captured", False) or getattr(gs, "inline", False)) and
                self.adam_ov is None and self.dadam is None)

    def _p_bwd_pair(self):
        if self.twin:
            self._bwd("p", self.pair, True)
        else:
            self._bwd("pr", self.pair, True)
            self._bwd("pl", self.pair, False)     # (backward ends by joining its filter-gradient stream)
        if self.grad_sync is not None and hasattr(self.grad_sync, "join"):
            self.grad_sync.join(self.pair.chunk)  # depth_net's exchange (branch joined / leftovers reduced) before its Adam
        if self._inline_adam():
            self.opt.opts[1].step()
            self._tl("pair adam")

    def _p_bwd_single(self):
        if self.twin:
            self._bwd("s", self.single, True)
        else:
            self._bwd("sr", self.single, True)
            self._bwd("sl", self.single, False)
        if self.grad_sync is not None and hasattr(self.grad_sync, "join"):
            self.grad_sync.join(self.single.chunk)
        if self._inline_adam():
            self.opt.opts[0].step()
            self._tl("single adam")

    def phase_compute(self):
        self._out = {}
        ov = self._overlap_stream()
        cur = torch.cuda.current_stream()
        fork = None
        for where, fn in self._pieces():
            if where == "join":
                if ov is not None:
                    _lib.wait_stream(cur, ov)
            elif where == "fork":
                if ov is not None:
                    fork = torch.cuda.Event()
                    fork.record(cur)
            elif where == "ov" and ov is not None:
                # depth_net on both pairs on the second stream, beside disp_net on both images
                if fork is not None:
                    _lib.wait_event(ov, fork)
                else:
                    _lib.wait_stream(ov, cur)
                with torch.cuda.stream(ov):
                    fn()
            else:
                fn()

    def _capture(self, warmup=2):
        """With the net overlap: one graph per piece, captured on the piece's stream; step() replays them
        with the same stream waits as the eager overlapped step.  (The whole step as ONE graph with depth_net's calls
        a forked branch measured no faster, round 3, and was removed in round 5.)"""
        if self._overlap_stream() is None:
            self.ov_seq = None
            return super()._capture(warmup)
        s = _lib.owned_stream(self, "capture_warmup")
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        main, ov = _lib.owned_stream(self, "capture"), self.net_stream
        gs = self.grad_sync
        seg = gs is not None and hasattr(gs, "begin_step") and not getattr(gs, "captured", False)
        pieces = self._pieces() + ([] if seg else [("main", self._update)])
        seq = []
        self._out = {}
        if gs is not None and hasattr(gs, "begin_step"):
            gs.begin_step()
        try:
            for where, fn in pieces:
                if where in ("join", "fork"):
                    seq.append((where, None))
                    continue
                stream = ov if where == "ov" else main
                # a piece is a list of graph segments: with the bucketed exchange, every bucket launch point of the
                # piece's backward closes the current segment (the program's filter-gradient branch joined first,
                # _join_chunk_wgrad); replay launches the buckets between segments, on the piece's stream
                segs = []
                state = {"g": torch.cuda.CUDAGraph()}

                def cut(buckets, state=state, segs=segs, stream=stream):
                    segs.append((_end_segment(state["g"]), list(buckets)))
                    state["g"] = torch.cuda.CUDAGraph()
                    state["g"].capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)

                with torch.cuda.stream(stream):
                    if seg:
                        gs.capturing = cut
                    state["g"].capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)
                    fn()
                    segs.append((_end_segment(state["g"]), []))
                seq.append((where, segs))
            if seg:
                gs.capturing = None
                leftovers = gs.leftovers()
                upd = None
                if not self._inline_adam():
                    # (over RCCL each chain's Adam follows its own exchange inline: no separate update graph)
                    upd = torch.cuda.CUDAGraph()
                    with torch.cuda.stream(main):
                        upd.capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)
                        self.phase_update()
                        upd.capture_end()
                self.ov_upd = (leftovers, upd)
        finally:
            if seg:
                gs.capturing = None
        torch.cuda.synchronize()
        self.ov_seq = seq
        self.graphs = [g for _, segs in seq if segs is not None for g, _ in segs if g is not None]
        if seg and self.ov_upd[1] is not None:
            self.graphs.append(self.ov_upd[1])
        return self.graphs

    def step(self):
        if self.graphs is None or getattr(self, "ov_seq", None) is None:
            return super().step()
        cur, ov = torch.cuda.current_stream(), self.net_stream
        gs = self.grad_sync
        seg = gs is not None and hasattr(gs, "begin_step") and not getattr(gs, "captured", False)
        if seg:
            gs.begin_step()
        fork = None
        for where, segs in self.ov_seq:
            if where == "join":
                cur.wait_stream(ov)
                continue
            if where == "fork":
                fork = torch.cuda.Event()
                fork.record(cur)
                continue
            if where == "ov":
                if fork is not None:
                    ov.wait_event(fork)
                else:
                    ov.wait_stream(cur)
            with torch.cuda.stream(ov if where == "ov" else cur):
                for g, buckets in segs:
                    if g is not None:
                        g.replay()
                    if buckets:
                        for b in buckets:
                            b.launched = True
                        gs.launch(buckets)      # the comm stream waits on this stream's tail
        if seg:
            gs.finish()
            if self.ov_upd[1] is not None:
                self.ov_upd[1].replay()

    def _p_loss(self):
        from . import losses as Ls
        lib, st = _lib.load(), _lib.stream_ptr()
        B, w, out = self.N, self.w, self._out
        # pose_final = reduce_mean(pose_pred, [1,2]) (nets_optflow_depth.py:183-186)
        pl, pr = out["pl"][4], out["pr"][4]
        hw = pl.shape[1] * pl.shape[2]
        if _halves(pl, pr):
            _lib.check(lib.tde_spatial_mean_fwd(2 * B, hw, 6, ptr(pl), 6, ptr(self.pose2), st), "pose mean")
        else:
            for pp, d in ((pl, "lr"), (pr, "rl")):
                _lib.check(lib.tde_spatial_mean_fwd(B, hw, 6, ptr(pp), 6, ptr(self.pose[d]), st), "pose mean")
        jobs = [dict(K=self.Ks[s], T=self.T[d] if s == 0 else None, P=self.P[d][s], Kinv=self.Kinv[s],
                     vec=self.pose[d]) for s in range(4) for d in ("lr", "rl")]
        Ls.pose_prep_multi(jobs)
        S = self.SLOTS
        _lib.check(lib.tde_cam_loss(B, ptr(self.gt_cam), ptr(self.T["lr"]), ptr(self.T["rl"]), w["cam"],
                                    Ls.dptr(self.acc, S["cam"]), ptr(self.gT["lr"]), ptr(self.gT["rl"]), st), "cam")
        # smoothness of 1/disp on the 4 maps at every scale (:216-225) and, on the single left net, the depth L1
        # to the area-downsampled label with replace_nonfinite (:227-232,241-243): depth_net's two maps in one
        # launch here, disp_net's two on its own chain (_p_fwd_single)
        Ls.pyramid_multi([self._pyramid_map(k) for k in ("pl", "pr")])   # disjoint gradient buffers
        dirs = (("l", "r", "pl", "pr", "lr"), ("r", "l", "pr", "pl", "rl"))
        calls = {d: [dict(img_src=self.pyr[src][s], img_tgt=self.pyr[tgt][s], P=self.P[d][s], Kinv=self.Kinv[s],
                          disp=out[run][s], logits=out[run][5 + s], disp_other=out[oth][s], photo_w=w["data"],
                          exp_w=w["exp"], consist_w=w["depth"], g_disp=self.d_out[run][s],
                          g_logits=self.d_out[run][5 + s], g_other=self.d_out[oth][s], g_P=self.gP[d][s],
                          det_ws=self.det_ws) for s in range(4)]
                 for tgt, src, run, oth, d in dirs}
        if self.det_ws is None:
            # one launch per direction over the 4 scales (a direction's calls write disjoint g_disp / g_logits;
            # the two directions of one scale do not: g_disp of one is g_other of the other)
            for d in ("lr", "rl"):
                Ls.warp_loss_multi(self.acc, S["photo"], calls[d])
        else:
            for s in range(4):
                for d in ("lr", "rl"):
                    Ls.warp_loss(self.acc, S["photo"], **calls[d][s])
        # pose gradients -> pose_pred (spatial mean backward)
        gl, gr = self.d_out["pl"][4], self.d_out["pr"][4]
        # both directions' pose gradients and their spatial-mean backward into the pose maps: one launch
        jobs = (_lib.PoseGradArgs * 2)()
        for j, (d, g) in enumerate((("lr", gl), ("rl", gr))):
            jobs[j] = _lib.PoseGradArgs(B, 4, ptr(self.pose[d]), ptr(self.K), 36, ptr(self.gP[d]), ptr(self.gT[d]),
                                        ptr(self.g_pose[d]), 0, ptr(g), hw, 6, 0)
        _lib.check(lib.tde_pose_grad_spread(jobs, 2, st), "pose grad spread")

    def loss_parts(self):
        v = self.acc.cpu().tolist()
        return {k: v[i] for k, i in self.SLOTS.items()}

    def total_loss(self):
        return float(sum(self.loss_parts().values()))


class OptflowCombineTrainer(Trainer):
    """Config 3: `train_optflow_combine.py` (canonical interpretation): joint
    depth + flow `nets_depth.disp_net` on concat(L,R) (:97-109); per scale (:138-237) smoothness of disp,
    flow-x, flow-y; depth L1; a ground-truth-depth warp giving wmask and the flow target (:169-176,205);
    wmask-weighted photometric L1 of the predicted-depth warp (:178-188) and of the flow warp
    (:191-198); flow L1 to depth_optflow (:205-210); pose is the given 4x4 tgt2src (format='matrix')."""

    SLOTS = dict(smooth=0, depth=1, photo=2, optflow=5)

    def __init__(self, batch, H=192, W=256, lr=2e-4, beta1=0.9, weights=None):
        from .losses import W_CONFIG3, Arena, new
        self.N, self.H, self.W = batch, H, W
        self.w = weights or W_CONFIG3
        with variables.variable_scope("model"):
            self.prog = _api.get_program("depth_net", _netlib.depthflow_net_spec, H, W, 6)
        self.chunks = [self.prog.chunk]
        self.opt = MultiAdam(self.chunks, lr, beta1)
        B = batch
        self.run = NetRun(self.prog, B)
        self.img = {"l": new((B, H, W, 3)), "r": new((B, H, W, 3))}
        self.pair_in = new((B, H, W, 6))
        self.label = new((B, H, W, 1))
        self.K = new((B, 4, 3, 3))
        self.tgt2src = new((B, 4, 4))
        self.pyr = {k: [self.img[k]] + [new(s) for s in _scale_shapes(B, H, W, 3)[1:]] for k in ("l", "r")}
        self.label_pyr = [self.label] + [new(s) for s in _scale_shapes(B, H, W, 1)[1:]]
        self.Ks = [new((B, 9)) for _ in range(4)]
        self.P = [new((B, 12)) for _ in range(4)]
        self.Kinv = [new((B, 9)) for _ in range(4)]
        self.wmask = [new((B, H >> s, W >> s)) for s in range(4)]
        self.gflow = [(new((B, H >> s, W >> s)), new((B, H >> s, W >> s))) for s in range(4)]
        # loss accumulators + the output gradients (the run's own gradient buffers): one arena, one zeroing
        ar = Arena()
        ia = ar.new((8,), torch.float64)
        ido = [ar.new((B, v.H, v.W, v.C)) for v in self.prog.spec.outputs]
        t = ar.finalize()
        self.arena, self.acc, self.d_out = ar, t[ia], [t[i] for i in ido]
        self.run.bind_output_grads(self.d_out)

    def set_batch(self, img_l, img_r, label, K, tgt2src):
        self.img["l"].copy_(img_l)
        self.img["r"].copy_(img_r)
        self.label.copy_(label)
        self.K.copy_(K)
        self.tgt2src.copy_(tgt2src)
        for s in range(4):
            self.Ks[s].copy_(self.K[:, s].reshape(-1, 9))

    def phase_update(self):
        self.opt.step()

    def phase_compute(self):
        from . import losses as Ls
        lib, st = _lib.load(), _lib.stream_ptr()
        B, H, W, w = self.N, self.H, self.W, self.w
        M = B * H * W
        self.arena.zero()
        _lib.check(lib.tde_copy_view(M, 3, ptr(self.img["l"]), 3, 0, ptr(self.pair_in), 6, 0, 0, st), "concat")
        _lib.check(lib.tde_copy_view(M, 3, ptr(self.img["r"]), 3, 0, ptr(self.pair_in), 6, 3, 0, st), "concat")
        out = self.prog.forward(self.run, self.pair_in)
        for s in range(1, 4):
            Ls.area(self.img["l"], self.pyr["l"][s])
            Ls.area(self.img["r"], self.pyr["r"][s])
            Ls.area(self.label, self.label_pyr[s])
        S = self.SLOTS
        # every scale's smoothness of disp (:143-144) with its depth L1 to the area-downsampled label
        # (:163-164), and of flow-x / flow-y (:147-150): one multi-scale launch each
        sw = [w["smooth"] / 2 ** s for s in range(4)]
        Ls.pyramid(out[:4], self.d_out[:4], self.acc, sw, S["smooth"], label=self.label,
                   l1_w=[w["depth"] / 2 ** s for s in range(4)], slot_l1=S["depth"])
        Ls.pyramid(out[4:8], self.d_out[4:8], self.acc, sw, S["smooth"], coff=0)
        Ls.pyramid(out[4:8], self.d_out[4:8], self.acc, sw, S["smooth"], coff=1)
        for s in range(4):
            disp, flow = out[s], out[4 + s]
            gd, gf = self.d_out[s], self.d_out[4 + s]
            ws = 1.0 / 2 ** s
            Ls.pose_prep(self.Ks[s], P=self.P[s], Kinv=self.Kinv[s], mat=self.tgt2src)
            h, wd = H >> s, W >> s
            _lib.check(lib.tde_warp_fwd(B, h, wd, 3, ptr(self.label_pyr[s]), 1, ptr(self.P[s]), ptr(self.Kinv[s]),
                                        None, None, 0, 0, None, None, ptr(self.gflow[s][0]), ptr(self.gflow[s][1]),
                                        ptr(self.wmask[s]), None, st), "gt warp")      # :169-176
            Ls.warp_loss(self.acc, S["photo"], self.pyr["r"][s], self.pyr["l"][s], P=self.P[s], Kinv=self.Kinv[s],
                         disp=disp, wmask=self.wmask[s], photo_w=w["data"] * ws, g_disp=gd,
                         det_ws=self.det_ws)                                            # :178-188
            Ls.warp_loss(self.acc, S["photo"], self.pyr["r"][s], self.pyr["l"][s], flow=flow, wmask=self.wmask[s],
                         photo_w=w["data"] * ws, g_flow=gf, det_ws=self.det_ws)         # :191-198
            Ls.l1(flow, self.gflow[s][0], gf, w["optflow"] * ws, self.acc, S["optflow"], coff=0)   # :205-207
            Ls.l1(flow, self.gflow[s][1], gf, w["optflow"] * ws, self.acc, S["optflow"], coff=1)   # :209-210
        # one backward call per step writes every parameter gradient: overwrite, no zeroed buffer
        self.prog.backward(self.run, [IN_PLACE] * len(self.d_out), on_grads=self.hook(self.prog.chunk),
                           grad_accumulate=False)

    def total_loss(self):
        return float(self.acc.sum().item())


class RefineTrainer(Trainer):
    """Config 5: `refine_depth.py` canonical interpretation: 1-channel sigmoid
    disp_net at 640x480; per scale (:185-213) smoothness of disp, |src - warp(tgt, 1/disp, pose)| and a
    depth L1 to the area-downsampled ground truth; fixed 4x4 pose, scale_factor = 1."""

    SLOTS = dict(smooth=0, depth=1, photo=2)

    def __init__(self, batch, H=480, W=640, lr=2e-5, beta1=0.9, weights=None):
        from .losses import W_CONFIG5, Arena, new
        self.N, self.H, self.W = batch, H, W
        self.w = weights or W_CONFIG5
        with variables.variable_scope("model"):
            self.prog = _api.get_program("depth_net", _netlib.disp_net_spec, H, W, 3, decay=0.99, scale=4.0,
                                         offset=0.0)
        self.chunks = [self.prog.chunk]
        self.opt = MultiAdam(self.chunks, lr, beta1)
        B = batch
        self.run = NetRun(self.prog, B)
        self.x1, self.x2 = new((B, H, W, 3)), new((B, H, W, 3))
        self.gt = new((B, H, W, 1))
        self.K = new((B, 4, 3, 3))
        self.pose = new((B, 4, 4))
        self.pyr1 = [self.x1] + [new(s) for s in _scale_shapes(B, H, W, 3)[1:]]
        self.pyr2 = [self.x2] + [new(s) for s in _scale_shapes(B, H, W, 3)[1:]]
        self.Ks = [new((B, 9)) for _ in range(4)]
        self.P = [new((B, 12)) for _ in range(4)]
        self.Kinv = [new((B, 9)) for _ in range(4)]
        ar = Arena()
        ia = ar.new((4,), torch.float64)
        ido = [ar.new((B, v.H, v.W, v.C)) for v in self.prog.spec.outputs]
        t = ar.finalize()
        self.arena, self.acc, self.d_out = ar, t[ia], [t[i] for i in ido]
        self.run.bind_output_grads(self.d_out)

    def set_batch(self, x1, x2, gt_disp, K, pose4):
        self.x1.copy_(x1)
        self.x2.copy_(x2)
        self.gt.copy_(gt_disp)
        self.K.copy_(K)
        self.pose.copy_(pose4)
        for s in range(4):
            self.Ks[s].copy_(self.K[:, s].reshape(-1, 9))

    def phase_update(self):
        self.opt.step()

    def phase_compute(self):
        from . import losses as Ls
        lib, st = _lib.load(), _lib.stream_ptr()
        self.arena.zero()
        out = self.prog.forward(self.run, self.x1)
        for s in range(1, 4):
            Ls.area(self.x1, self.pyr1[s])
            Ls.area(self.x2, self.pyr2[s])
        S, w = self.SLOTS, self.w
        # every scale's smoothness (:186-187) and depth L1 to the area-downsampled ground truth (:210-213):
        # one multi-scale launch
        Ls.pyramid(out[:4], self.d_out[:4], self.acc, [w["smooth"] / 2 ** s for s in range(4)], S["smooth"],
                   label=self.gt, l1_w=[w["data"] / 2 ** s for s in range(4)], slot_l1=S["depth"])
        for s in range(4):
            disp, g = out[s], self.d_out[s]
            Ls.pose_prep(self.Ks[s], P=self.P[s], Kinv=self.Kinv[s], mat=self.pose)
            Ls.warp_loss(self.acc, S["photo"], self.pyr2[s], self.pyr1[s], P=self.P[s], Kinv=self.Kinv[s],
                         disp=disp, photo_w=1.0, g_disp=g, det_ws=self.det_ws)              # :200-212
        # one backward call per step writes every parameter gradient: overwrite, no zeroed buffer
        self.prog.backward(self.run, [IN_PLACE] * len(self.d_out), on_grads=self.hook(self.prog.chunk),
                           grad_accumulate=False)

    def total_loss(self):
        return float(self.acc.sum().item())
