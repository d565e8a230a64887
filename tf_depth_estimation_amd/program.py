"""Layer-program executor: a static schedule of C-ABI kernel calls for one encoder/decoder network.

The reference builds each network as a TF-1 graph of slim layers (nets_optflow_depth.py:76-276,
nets_depth.py:76-199).  Here a network is built once per (input H, W) into a `NetSpec`: a list of ops
over *channel views* of NHWC activation buffers.  tf.concat(axis=3) is never materialised: each
producer writes its result straight into its channel slice of the consumer's buffer, and the
consumer's implicit-GEMM reads the whole buffer (include/tde.h "channel view").  Concat buffers whose
width is not a multiple of 4 (e.g. 64+64+1 = 129 for icnv3) are zero-padded to 4 so every conv
operand is a 16-byte vector; the padded weight rows read as zero (`w_cin`).

Backward is the reverse schedule: for every op, the gradient of its output view is complete when it
is reached (all consumers come later in forward order), and the op writes (first writer) or
accumulates (later writers) into the gradient view of its input.  Parameter gradients always
accumulate into the ParamChunk's flat gradient buffer, which the trainer zeroes once per step, so a
network called twice with shared variables (train_depth_then_cam_lr.py:130-136) sums both calls like
TF does.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import ConvDesc, ptr


def same_pad(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return out, tot // 2


def pad4(c):
    return (c + 3) // 4 * 4


class Buf:
    def __init__(self, name, H, W, cs, zero=False):
        self.name, self.H, self.W, self.cs, self.zero = name, H, W, cs, zero


class View:
    def __init__(self, buf, coff, C, creal=None):
        self.buf, self.coff, self.C = buf, coff, C
        self.creal = C if creal is None else creal

    @property
    def H(self):
        return self.buf.H

    @property
    def W(self):
        return self.buf.W


class Op:
    params = ()
    branch = 0      # 1: a side branch of the network (depth_net's pose / mask heads: a timeline label only)


class ConvBN(Op):
    """slim.conv2d / slim.conv2d_transpose with normalizer_fn=batch_norm (+ReLU); or, with bn=False,
    with bias (+ReLU) as in the BN-free pairtest disp_net (nets_optflow_depth_pairtest.py:83-85)."""

    def __init__(self, layer, src, dst, K, k, s, deconv=False, bn=True, decay=0.99):
        self.layer, self.src, self.dst, self.K, self.k, self.s = layer, src, dst, K, k, s
        self.deconv, self.bn, self.decay = deconv, bn, decay
        cin = src.creal
        if deconv:
            # virtual forward conv: x = deconv output (dst, 2h x 2w x K), y = deconv input (src)
            self.OH, self.OW = src.H, src.W
            H, W = dst.H, dst.W
            _, self.pt = same_pad(H, k, s)
            _, self.pl = same_pad(W, k, s)
            wshape = (k, k, K, cin)
        else:
            self.OH, self.pt = same_pad(src.H, k, s)
            self.OW, self.pl = same_pad(src.W, k, s)
            wshape = (k, k, cin, K)
        assert (dst.H, dst.W) == ((src.H * s, src.W * s) if deconv else (self.OH, self.OW)), layer
        self.params = [(f"{layer}/weights", wshape, "glorot")]
        if bn:
            self.params.append((f"{layer}/BatchNorm/beta", (K,), "zeros"))
            self.bn_stats = [(f"{layer}/BatchNorm", K)]
        else:
            self.params.append((f"{layer}/biases", (K,), "zeros"))
            self.bn_stats = []

    def desc(self, N):
        d = ConvDesc()
        if self.deconv:
            d.N, d.H, d.W, d.C = N, self.dst.H, self.dst.W, self.K
            d.OH, d.OW, d.K = self.src.H, self.src.W, self.src.C
            d.w_cin = self.K
            d.x_cstride, d.x_coff = self.K, 0                       # dense pre-BN z (big)
            d.y_cstride, d.y_coff = self.src.buf.cs, self.src.coff  # deconv input view
        else:
            d.N, d.H, d.W, d.C = N, self.src.H, self.src.W, self.src.C
            d.OH, d.OW, d.K = self.OH, self.OW, self.K
            d.w_cin = self.src.creal
            d.x_cstride, d.x_coff = self.src.buf.cs, self.src.coff
            d.y_cstride, d.y_coff = self.K, 0                       # dense pre-BN z
        d.KH = d.KW = self.k
        d.stride, d.pad_top, d.pad_left = self.s, self.pt, self.pl
        return d

    def zshape(self, N):
        return (N, self.dst.H, self.dst.W, self.K)

    def folded_desc(self, N):
        """desc() with the output going straight into the consumer's channel view (folded-BN
        inference: no pre-BN z)."""
        d = self.desc(N)
        if self.deconv:
            d.x_cstride, d.x_coff = self.dst.buf.cs, self.dst.coff
        else:
            d.y_cstride, d.y_coff = self.dst.buf.cs, self.dst.coff
        return d


class Head(Op):
    """slim.conv2d(normalizer_fn=None) head with bias: act 1 -> scale*sigmoid(.)+offset, 0 -> linear."""

    def __init__(self, layer, src, dst, K, k, act, scale=1.0, offset=0.0):
        self.layer, self.src, self.dst, self.K, self.k = layer, src, dst, K, k
        self.act, self.scale, self.offset = act, scale, offset
        _, self.pt = same_pad(src.H, k, 1)
        _, self.pl = same_pad(src.W, k, 1)
        self.params = [(f"{layer}/weights", (k, k, src.creal, K), "glorot"), (f"{layer}/biases", (K,), "zeros")]
        self.bn_stats = []

    def desc(self, N):
        d = ConvDesc()
        d.N, d.H, d.W, d.C = N, self.src.H, self.src.W, self.src.C
        d.OH, d.OW, d.K = self.src.H, self.src.W, self.K
        d.KH = d.KW = self.k
        d.stride, d.pad_top, d.pad_left = 1, self.pt, self.pl
        d.w_cin = self.src.creal
        d.x_cstride, d.x_coff = self.src.buf.cs, self.src.coff
        d.y_cstride, d.y_coff = self.dst.buf.cs, self.dst.coff
        return d


class Resize(Op):
    """tf.image.resize_nearest_neighbor (resize_like) or resize_bilinear, legacy semantics."""

    def __init__(self, kind, src, dst):
        self.kind, self.src, self.dst = kind, src, dst
        self.bn_stats = []


class Copy(Op):
    """Second placement of a tensor that two concats consume (nets_depth.py shares the encoder)."""

    def __init__(self, src, dst):
        self.src, self.dst = src, dst
        self.bn_stats = []


class NetSpec:
    """Builder used by the per-net modules (nets_optflow_depth.py etc.)."""

    def __init__(self, scope, H, W, cin):
        self.scope, self.H, self.W, self.cin = scope, H, W, cin
        self.bufs, self.ops, self.outputs = [], [], []
        self.input = self.buffer("input", H, W, pad4(cin), zero=True)
        self.input_view = View(self.input, 0, pad4(cin), cin)

    def buffer(self, name, H, W, cs, zero=False):
        b = Buf(name, H, W, cs, zero)
        self.bufs.append(b)
        return b

    def concat(self, name, H, W, widths):
        """Allocate a concat buffer; returns its slice views and the full (padded) view."""
        total = sum(widths)
        cs = pad4(total)
        b = self.buffer(name, H, W, cs, zero=(cs != total))
        views, off = [], 0
        for w in widths:
            views.append(View(b, off, w))
            off += w
        return views, View(b, 0, cs, total)

    def dense(self, name, H, W, C):
        return View(self.buffer(name, H, W, C), 0, C)

    def add(self, op):
        self.ops.append(op)
        return op

    def param_specs(self):
        seen, specs, bn = set(), [], []
        for op in self.ops:
            for p in op.params:
                if p[0] not in seen:
                    seen.add(p[0])
                    specs.append(p)
            for b in op.bn_stats:
                bn.append(b)
        return specs, bn


SERIAL = "serial"   # enable_wgrad_overlap(serial=True): the split backward calls on the compute stream
# forward(run, IN_PLACE): the input is already in run.input_tensor(); backward(run, [IN_PLACE, ...]): that
# output's gradient was already written into run.grad_tensor(view) (e.g. by a loss kernel), so the step skips
# the copy launches
IN_PLACE = "in_place"


class Workspace:
    """Per-(program, batch) scratch shared by all calls on one stream: the split-K / reduction workspace
    and the dense dz buffer of the BN backward."""

    def __init__(self):
        self.ws = None
        self.dz = None

    def get(self, ws_bytes, dz_numel, device):
        if self.ws is None or self.ws.numel() * 4 < ws_bytes:
            self.ws = torch.empty(max(ws_bytes // 4 + 64, 64), dtype=torch.float32, device=device)
        if self.dz is None or self.dz.numel() < dz_numel:
            self.dz = torch.empty(max(dz_numel, 4), dtype=torch.float32, device=device)
        return self.ws, self.dz


class NetRun:
    """Per-invocation state of a program: activations, pre-BN outputs and batch statistics (the
    'tape' the backward pass needs).

    groups G > 1: the batch holds G equal consecutive sub-batches that are G separate calls of the network in the
    reference (shared variables, separate BatchNorm batches: disp_net on the left and on the right image,
    train_depth_then_cam_lr.py:130-136).  Every conv runs ONCE over all N rows (weights shared, twice the rows of
    the deep levels' GEMMs in one launch), every BatchNorm normalises each sub-batch over its own rows (tde_bn_*
    groups), and one backward call yields the sum of the calls' parameter gradients -- what TF computes for the
    shared variables."""

    def __init__(self, prog, N, device="cuda", groups=1):
        if groups < 1 or N % groups:
            raise ValueError(f"batch {N} is not {groups} equal groups")
        self.prog, self.N, self.device, self.groups = prog, N, device, groups
        self.act = {}
        for b in prog.spec.bufs:
            shape = (N, b.H, b.W, b.cs)
            self.act[b.name] = (torch.zeros(shape, device=device, dtype=torch.float32) if b.zero
                                else torch.empty(shape, device=device, dtype=torch.float32))
        self.z, self.stats = {}, {}
        for i, op in enumerate(prog.spec.ops):
            if isinstance(op, ConvBN) and op.bn:
                self.z[i] = torch.empty(op.zshape(N), device=device, dtype=torch.float32)
                self.stats[i] = torch.empty((2, groups * op.K), device=device, dtype=torch.float32)
            elif isinstance(op, ConvBN):
                self.z[i] = None
        # per-op bound max|dz| of the BN backward's output (tde_bn_bwd dz_absmax), the gradient operand bound
        # of the conv backward in fp16x3 conv math (tde_conv_desc_t); zeroed at the start of every backward
        self.absmax = torch.zeros((max(len(prog.spec.ops), 1), _lib.BOUND_SLOTS), device=device, dtype=torch.float32)
        self.grad = None

    def vptr(self, v, grad=False):
        t = (self.grad if grad else self.act)[v.buf.name]
        return ptr(t)

    def absmax_ptr(self, i):
        return self.absmax[i].data_ptr()

    def view_tensor(self, v, grad=False):
        t = (self.grad if grad else self.act)[v.buf.name]
        return t[..., v.coff:v.coff + v.C]

    def ensure_grad(self):
        if self.grad is None:
            self.grad = {b.name: torch.empty((self.N, b.H, b.W, b.cs), device=self.device, dtype=torch.float32)
                         for b in self.prog.spec.bufs}
        return self.grad

    def bind_output_grads(self, tensors):
        """Use the given dense [N,H,W,cs] tensors as the gradient buffers of the program's output buffers
        (e.g. views of one per-step arena that a trainer zeroes with one launch and its loss kernels write);
        backward(run, [IN_PLACE, ...]) then reads them where they are."""
        self.ensure_grad()
        for v, t in zip(self.prog.spec.outputs, tensors):
            b = v.buf
            if v.coff != 0 or v.C != b.cs or tuple(t.shape) != (self.N, b.H, b.W, b.cs) or not t.is_contiguous():
                raise ValueError(f"output {b.name}: needs a dense [N,H,W,{b.cs}] tensor")
            self.grad[b.name] = t

    def input_tensor(self):
        """The input view [N,H,W,cin] of the program's input buffer (write the batch here and call
        forward(run, IN_PLACE) to skip the input copy)."""
        iv = self.prog.spec.input_view
        return self.act[iv.buf.name][..., iv.coff:iv.coff + self.prog.spec.cin]

    def grad_tensor(self, v):
        """Gradient view of output view v (a loss kernel may write it; then pass IN_PLACE to backward)."""
        self.ensure_grad()
        return self.view_tensor(v, True)


class NetProgram:
    """Compiled network: spec + parameter chunk + launch schedule (forward and backward)."""

    def __init__(self, spec, chunk, bessel=True):
        self.spec, self.chunk, self.bessel = spec, chunk, bessel
        self.prefix = chunk.prefix
        self._ws = {}
        self._sizes = {}
        self.timer = None
        # SyncBN: bn_sync(t) all-reduces (sums) a float64 device tensor in place across
        # bn_world data-parallel replicas; None = BatchNorm over the local batch (the default)
        self.bn_sync, self.bn_world = None, 1
        self._bn_sums = {}
        self._folded = None     # layer -> (weights with BN folded in, bias); see fold_bn()
        # filter-gradient overlap (enable_wgrad_overlap): side stream, its workspace per batch, dz ring
        # (every conv layer but the first of forward sends its filter gradient to the side stream, each behind one event,
        # and the heads' filter gradients join it; measured and removed in round 5: groups of 2-3 layers per wait,
        # 2-3 tail layers inline, the deep layers inline, two side streams -- all equal or slower)
        self.wgrad_stream = None
        self._ws2 = {}
        self._dzl = {}
        self._wsplit = {}       # (N, conv math) -> pre-split weight images (_split_plan)
        self._cur_split = None
        self._spans = {}
        # forward hooks (Trainer.enable_deferred_adam): pre_op(prog, i) orders the current stream after
        # whatever updates op i's parameters; params_ready(prog, i) tells whether that has been done
        self.pre_op = None
        self.params_ready = None
        self.pre_backward = None    # called first thing in backward (before any gradient is written)
        self.timeline = None        # StepTimeline (diagnostic): a device stamp after every op, under capture only

    def _split_plan(self, N):
        """The convs whose forward or data-gradient call takes the halo-tiled path (their weights are kept as
        split MFMA tiles, tde_conv2d_split_weights): [(op index, op, desc, buffer)], cached per (N, conv math)."""
        lib = _lib.load()
        key = (N, lib.tde_get_conv_math())
        plan = self._wsplit.get(key)
        if plan is None:
            plan = []
            for i, op in enumerate(self.spec.ops):
                if not isinstance(op, ConvBN):
                    continue
                d = op.desc(N)
                for o in (0, 1):
                    # op code o + 2 for a deconv: the size of the image the calls of that role read (include/tde.h)
                    oc = o | (2 if op.deconv else 0)
                    nb = lib.tde_conv2d_split_weights_size(ctypes_ref(d), oc)
                    if nb:
                        plan.append((i, o, d, torch.empty((nb + 255) // 256 * 64, dtype=torch.float32, device="cuda"),
                                     oc))
            self._wsplit[key] = plan
        return key, plan

    def _issue_split(self, jobs):
        """Split the weights of `jobs` (entries of _split_plan) in ONE launch; valid until the weights change
        (the optimizer step): the forward makes them, and the backward of that forward uses them."""
        if not jobs:
            return
        lib = _lib.load()
        n = len(jobs)
        descs = (ctypes.c_void_p * n)(*[ctypes.addressof(d) for _, _, d, _, _ in jobs])
        ops = (ctypes.c_int * n)(*[oc for _, _, _, _, oc in jobs])
        ws = (ctypes.c_void_p * n)(*[self.P(f"{self.spec.ops[i].layer}/weights").data_ptr() for i, _, _, _, _ in jobs])
        outs = (ctypes.c_void_p * n)(*[t.data_ptr() for _, _, _, t, _ in jobs])
        _lib.check(lib.tde_conv2d_split_weights(n, descs, ops, ws, outs, _lib.stream_ptr()), "split weights")
        for i, o, _, t, _ in jobs:
            self._cur_split[1].setdefault(i, [None, None])[o] = t.data_ptr()

    def op_param_span(self, i):
        """[lo, hi) flat-buffer span of op i's parameters (None without parameters)."""
        span = self._spans.get(i)
        if span is None and i not in self._spans:
            op = self.spec.ops[i]
            names = [f"{self.prefix}/{n}" for n, _, _ in getattr(op, "params", [])]
            if names:
                lo = min(self.chunk.offsets[n] for n in names)
                hi = max(self.chunk.offsets[n] + int(np.prod(self.chunk.shapes[n])) for n in names)
                span = (lo, hi)
            self._spans[i] = span
        return span

    def _use_split(self, d, i, N):
        cur = getattr(self, "_cur_split", None)
        if cur is not None and cur[0] == (N, _lib.load().tde_get_conv_math()):
            sp = cur[1].get(i)
            if sp is not None:
                d.w_split[0], d.w_split[1] = sp[0], sp[1]

    def _sums(self, i, K, which, G=1):
        """fp64 per-channel sums [G][2K] of op i (which: 0 forward, 1 local backward, 2 all-reduced backward)."""
        key = (i, which, G)
        t = self._bn_sums.get(key)
        if t is None:
            t = self._bn_sums[key] = torch.empty((G, 2 * K), dtype=torch.float64, device="cuda")
        return t

    def _span(self, family, flops=0.0, nbytes=0.0):
        return NO_SPAN if self.timer is None else self.timer.span(family, flops, nbytes)

    def _production(self):
        """The shipped schedule runs (fused conv + BN calls, filter gradients on their side stream): no timer, or a
        GraphTimer (which times that schedule where a captured graph replays it); a KernelTimer's instrumented eager
        step instead splits conv and BN calls and keeps one stream."""
        return self.timer is None or getattr(self.timer, "graph", False)

    # ---------------------------------------------------------------- helpers
    def P(self, name):
        return self.chunk.view(f"{self.prefix}/{name}")

    def G(self, name):
        return self.chunk.grad_view(f"{self.prefix}/{name}")

    def fold_bn(self):
        """Inference weights: each conv/deconv's moving statistics folded into its weights and a bias
        (tde_bn_fold; batch_prediction.py:41-44 runs disp_net with is_training=False).  A snapshot of the
        current variables: call again after a checkpoint restore or further training."""
        fl = getattr(self.chunk, "pending_flush", None)
        if fl is not None:
            fl()            # a deferred-Adam trainer's owed update first (Trainer.flush)
        lib = _lib.load()
        st = _lib.stream_ptr()
        folded = {}
        for op in self.spec.ops:
            if not (isinstance(op, ConvBN) and op.bn):
                continue     # (BN-free layers run their own weights and biases)
            w = self.P(f"{op.layer}/weights")
            beta = self.P(f"{op.layer}/BatchNorm/beta")
            mm, mv = self.chunk.moving(f"{self.prefix}/{op.layer}/BatchNorm")
            kh, kw, a, b = w.shape
            layout, cin = (1, b) if op.deconv else (0, a)
            wf = torch.empty_like(w)
            bf = torch.empty(op.K, dtype=torch.float32, device=w.device)
            _lib.check(lib.tde_bn_fold(kh * kw, cin, op.K, layout, ptr(w), ptr(mm), ptr(mv), ptr(beta), 1e-3,
                                       ptr(wf), ptr(bf), st), op.layer + " fold")
            # folded weights are w * rsqrt(moving_var + eps): their bound for the fp16x3 split (a layer with a
            # small moving variance can exceed the fixed 2^8 weight scale's range)
            wb = torch.zeros(_lib.BOUND_SLOTS, dtype=torch.float32, device=w.device)
            wb[0] = wf.abs().amax()
            folded[op.layer] = (wf, bf, wb)
        self._folded = folded
        return folded

    def enable_wgrad_overlap(self, on=True, serial=False):
        """Take the filter gradients off backward's critical path: each conv/deconv's data gradient runs on
        the current stream and its filter gradient (tde_conv2d_bwd_filter / tde_deconv2d_bwd_filter) on a side
        stream, with its own workspace.  Every layer's BN backward writes its own dz buffer, so nothing on the
        data-gradient chain ever waits for a filter gradient (TF's Conv2DBackpropFilter has no consumer but
        the optimizer): the side stream only waits for the compute stream, once per conv layer (one event),
        and under capture it is a parallel graph branch joined at the end of backward (and before
        any gradient-exchange launch point: join_wgrad()).  The two GEMMs are the separate data- and
        filter-gradient calls (their own tile plans, not the fused launch's shared tile), so results equal
        serial=True -- the same calls in the same order on ONE stream -- bit for bit."""
        # dedicated HIP streams, one per role and program (torch.cuda.Stream() recycles a fixed pool: a pooled
        # side stream can alias a capture stream or another program's side stream, _lib.dedicated_stream)
        self.wgrad_stream = (SERIAL if serial else _lib.owned_stream(self, "wgrad0")) if on else None
        self.wgrad_streams = [self.wgrad_stream] if on else []
        self._wg_rr = 0
        return self

    def join_wgrad(self):
        """Order the current stream after every filter gradient launched so far (the dz ring is then free:
        its events are dropped, so none is waited on across a graph-segment boundary)."""
        if self.wgrad_stream is not None:
            self._flush_wgrad()
            if self.wgrad_stream is not SERIAL:
                for sd in self.wgrad_streams:
                    _lib.wait_stream(torch.cuda.current_stream(), sd)

    def _flush_wgrad(self, ev=None):
        """Issue the deferred filter gradients on the side stream behind ONE wait for the compute stream: on
        `ev` (recorded on it after the last of their dz was written) or on everything issued so far."""
        pending = getattr(self, "_wg_pending", None)
        if not pending:
            return
        side = self.wgrad_stream
        sidx = 0
        if side is SERIAL:
            side = torch.cuda.current_stream()
        else:
            sidx = self._wg_rr % len(self.wgrad_streams)
            self._wg_rr += 1
            side = self.wgrad_streams[sidx]
            if ev is not None:
                _lib.wait_event(side, ev)
            else:
                _lib.wait_stream(side, torch.cuda.current_stream())
        ws2 = self._scratch_side(self._wg_N, sidx)
        with torch.cuda.stream(side):
            for fn, _ in pending:
                fn(ptr(ws2), ws2.numel() * 4)
        self._wg_issued.extend(n for _, names in pending for n in names)
        pending.clear()

    def _scratch_side(self, N, sidx=0):
        ws, _ = self._scratch(N)
        w = self._ws2.setdefault((N, sidx), Workspace())
        return w.get(ws.numel() * 4, 4, "cuda")[0]

    def _dz_layer(self, N, i, numel):
        """Layer i's own dz buffer (filter-gradient overlap): never reused within a backward call, so the
        BN backward never waits for the filter gradient that reads it."""
        t = self._dzl.get((N, i))
        if t is None or t.numel() < numel:
            t = self._dzl[(N, i)] = torch.empty(max(numel, 4), dtype=torch.float32, device="cuda")
        return t

    def _scratch(self, N):
        if N not in self._sizes:
            lib = _lib.load()
            ws, dz = 0, 0
            for op in self.spec.ops:
                if isinstance(op, ConvBN):
                    d = op.desc(N)
                    q = lib.tde_deconv2d_workspace_size if op.deconv else lib.tde_conv2d_workspace_size
                    for o in range(4):
                        ws = max(ws, q(ctypes_ref(d), o))
                    qb = lib.tde_deconv2d_bwd_workspace_size if op.deconv else lib.tde_conv2d_bwd_workspace_size
                    ws = max(ws, qb(ctypes_ref(d)))
                    ws = max(ws, q(ctypes_ref(op.folded_desc(N)), 1 if op.deconv else 0))
                    M = N * op.dst.H * op.dst.W
                    ws = max(ws, lib.tde_bn_workspace_size(M, op.K))
                    dz = max(dz, M * op.K)
                elif isinstance(op, Head):
                    ws = max(ws, lib.tde_head_workspace_size(ctypes_ref(op.desc(N))))
            self._sizes[N] = (ws, dz)
        ws, dz = self._sizes[N]
        w = self._ws.setdefault(N, Workspace())
        return w.get(ws, dz, "cuda")

    # ---------------------------------------------------------------- forward
    def forward(self, run, x, is_training=True, fold_bn=False):
        """x: [N,H,W,cin] fp32 on the device.  Returns the output view tensors.  fold_bn (inference only):
        run each conv/deconv + BN + ReLU as ONE bias+ReLU conv on the weights of fold_bn()."""
        main = torch.cuda.current_stream()
        try:
            return self._forward(run, x, is_training, fold_bn)
        finally:
            torch.cuda.set_stream(main)

    def _forward(self, run, x, is_training, fold_bn):
        if fold_bn and (is_training or self._folded is None):
            raise ValueError("fold_bn needs is_training=False and weights folded by fold_bn()")
        N = run.N
        lib = _lib.load()
        st = _lib.stream_ptr()
        spec = self.spec
        iv = spec.input_view
        if not (isinstance(x, str) and x == IN_PLACE):
            assert tuple(x.shape) == (N, spec.H, spec.W, spec.cin), (x.shape, spec.H, spec.W, spec.cin)
            x = x.contiguous()
            _lib.check(lib.tde_copy_view(N * spec.H * spec.W, spec.cin, ptr(x), spec.cin, 0, run.vptr(iv), iv.buf.cs,
                                         0, 0, st), "copy input")
        ws, _ = self._scratch(N)
        wsb = ws.numel() * 4
        split_todo = {}
        if fold_bn:
            self._cur_split = None
        else:
            key, plan = self._split_plan(N)
            self._cur_split = (key, {})
            for job in plan:
                split_todo.setdefault(job[0], []).append(job)
        tl = self.timeline
        for i, op in enumerate(spec.ops):
            if tl is not None and i > 0:
                tl.mark(self.prefix, "F", spec.ops[i - 1])
            if self.timer is not None:
                self.timer.tag = getattr(op, "layer", type(op).__name__)
            if self.pre_op is not None and isinstance(op, (ConvBN, Head)):
                self.pre_op(self, i)
            if isinstance(op, ConvBN):
                if i in split_todo:
                    # one split launch for every pending layer whose weights are final by now (all of them
                    # unless an optimizer step is still running on a side stream)
                    ready = [j for j in split_todo if self.params_ready is None or self.params_ready(self, j)]
                    self._issue_split([job for j in ready for job in split_todo.pop(j)])
                d = op.desc(N)
                if not fold_bn:
                    self._use_split(d, i, N)
                w = self.P(f"{op.layer}/weights")
                z = run.z[i] if op.bn else None
                if not op.bn:
                    # BN-free layer (nets_optflow_depth_pairtest.py:83-85): conv + bias + ReLU in one launch,
                    # written straight into the consumer's channel view (training and inference alike)
                    fd = op.folded_desc(N)
                    if not fold_bn:
                        self._use_split(fd, i, N)
                    fn = lib.tde_deconv2d_fwd_bias_act if op.deconv else lib.tde_conv2d_fwd_bias_act
                    with self._span("conv_fwd", conv_flops(op, N), conv_bytes(op, N)):
                        _lib.check(fn(ctypes_ref(fd), run.vptr(op.src), ptr(w), ptr(self.P(f"{op.layer}/biases")), 1,
                                      run.vptr(op.dst), ptr(ws), wsb, st), op.layer)
                    continue
                M = N * op.dst.H * op.dst.W
                beta = self.P(f"{op.layer}/BatchNorm/beta")
                sm = run.stats[i]
                mm, mv = self.chunk.moving(f"{self.prefix}/{op.layer}/BatchNorm")
                if fold_bn:
                    wf, bf, wb = self._folded[op.layer]
                    fd = op.folded_desc(N)
                    fd.w_absmax = wb.data_ptr()
                    fn = lib.tde_deconv2d_fwd_bias_act if op.deconv else lib.tde_conv2d_fwd_bias_act
                    with self._span("conv_fwd", conv_flops(op, N), conv_bytes(op, N)):
                        _lib.check(fn(ctypes_ref(fd), run.vptr(op.src), ptr(wf), ptr(bf), 1, run.vptr(op.dst), ptr(ws),
                                      wsb, st), op.layer)
                elif is_training and self.bn_sync is not None:
                    # SyncBN: the conv writes its local (sum z, sum z^2) per row group from its own statistics
                    # partials, ONE all-reduce of all groups' sums, then one apply launch normalises each group over its
                    # rows of all replicas (a twin run's left / right halves stay separate BatchNorm batches, as the
                    # reference's two calls, train_depth_then_cam_lr.py:130-136)
                    G = run.groups
                    Mg = M // G
                    sums = self._sums(i, op.K, 0, G)
                    bn = _lib.BnTrain(ptr(beta), 1e-3, op.decay, int(self.bessel), ptr(mm), ptr(mv), ptr(sm[0]),
                                      ptr(sm[1]), run.vptr(op.dst), op.dst.buf.cs, op.dst.coff, 1, G, ptr(sums))
                    fn = lib.tde_deconv2d_fwd_bn if op.deconv else lib.tde_conv2d_fwd_bn
                    _lib.check(fn(ctypes_ref(d), run.vptr(op.src), ptr(w), ptr(z), ctypes_ref(bn), ptr(ws), wsb, st),
                               op.layer + " bn sums")
                    self.bn_sync(sums)
                    _lib.check(lib.tde_bn_fwd_from_sums(M, op.K, G, Mg * self.bn_world, ptr(z), ptr(sums), ptr(beta),
                                                        1e-3, op.decay, int(self.bessel), ptr(mm), ptr(mv), ptr(sm[0]),
                                                        ptr(sm[1]), run.vptr(op.dst), op.dst.buf.cs, op.dst.coff, 1, st),
                               op.layer + " syncbn")
                elif is_training and self._production():
                    # conv + batch norm (batch statistics, moving averages) + ReLU: one ABI call; the BN pass
                    # consumes the conv's split-K partials directly (a GraphTimer times its conv kernels only)
                    bn = _lib.BnTrain(ptr(beta), 1e-3, op.decay, int(self.bessel), ptr(mm), ptr(mv), ptr(sm[0]),
                                      ptr(sm[1]), run.vptr(op.dst), op.dst.buf.cs, op.dst.coff, 1, run.groups)
                    fn = lib.tde_deconv2d_fwd_bn if op.deconv else lib.tde_conv2d_fwd_bn
                    with self._span("conv_fwd", conv_flops(op, N), conv_bytes(op, N)):
                        _lib.check(fn(ctypes_ref(d), run.vptr(op.src), ptr(w), ptr(z), ctypes_ref(bn), ptr(ws), wsb,
                                      st), op.layer)
                elif is_training:
                    # instrumented step (bench.py roofline): the same layer as separate conv and BN calls, so
                    # the conv kernel's time is measured on its own
                    fn = lib.tde_deconv2d_fwd if op.deconv else lib.tde_conv2d_fwd
                    with self._span("conv_fwd", conv_flops(op, N), conv_bytes(op, N)):
                        _lib.check(fn(ctypes_ref(d), run.vptr(op.src), ptr(w), ptr(z), 0, ptr(ws), wsb, st), op.layer)
                    with self._span("bn_fwd"):
                        _lib.check(lib.tde_bn_fwd_train(M, op.K, run.groups, ptr(z), ptr(beta), 1e-3, op.decay,
                                                        int(self.bessel),
                                                        ptr(mm), ptr(mv), ptr(sm[0]), ptr(sm[1]), run.vptr(op.dst),
                                                        op.dst.buf.cs, op.dst.coff, 1, ptr(ws), wsb, st), op.layer)
                else:
                    fn = lib.tde_deconv2d_fwd if op.deconv else lib.tde_conv2d_fwd
                    with self._span("conv_fwd", conv_flops(op, N), conv_bytes(op, N)):
                        _lib.check(fn(ctypes_ref(d), run.vptr(op.src), ptr(w), ptr(z), 0, ptr(ws), wsb, st), op.layer)
                    with self._span("bn_fwd"):
                        _lib.check(lib.tde_bn_fwd_infer(M, op.K, ptr(z), ptr(beta), 1e-3, ptr(mm), ptr(mv),
                                                        run.vptr(op.dst), op.dst.buf.cs, op.dst.coff, 1, st), op.layer)
            elif isinstance(op, Head):
                d = op.desc(N)
                with self._span("head_fwd", conv_flops(op, N)):
                    _lib.check(lib.tde_head_fwd(ctypes_ref(d), run.vptr(op.src), ptr(self.P(f"{op.layer}/weights")),
                                                ptr(self.P(f"{op.layer}/biases")), run.vptr(op.dst), op.act, op.scale,
                                                op.offset, st), op.layer)
            elif isinstance(op, Resize):
                s, t = op.src, op.dst
                fn = lib.tde_resize_nearest_fwd if op.kind == "nearest" else lib.tde_resize_bilinear_fwd
                with self._span("resize"):
                    _lib.check(fn(N, s.H, s.W, s.C, run.vptr(s), s.buf.cs, s.coff, t.H, t.W, run.vptr(t), t.buf.cs,
                                  t.coff, st), op.kind)
            elif isinstance(op, Copy):
                s, t = op.src, op.dst
                _lib.check(lib.tde_copy_view(N * s.H * s.W, s.C, run.vptr(s), s.buf.cs, s.coff, run.vptr(t),
                                             t.buf.cs, t.coff, 0, st), "copy")
        if tl is not None and spec.ops:
            tl.mark(self.prefix, "F", spec.ops[-1])
        return [run.view_tensor(v) for v in spec.outputs]

    # ---------------------------------------------------------------- backward
    def backward(self, run, grad_outputs, need_input_grad=False, on_grads=None, grad_accumulate=True):
        """grad_outputs: list (aligned with spec.outputs) of tensors or None.  Accumulates parameter
        gradients into chunk.grad, or with grad_accumulate=False OVERWRITES them (every parameter is
        written by one backward call, so a trainer's first call of the step needs no zeroed buffer
        and the kernels skip the read-modify-write).  Returns d(input) if requested.  on_grads(names),
        if given, is called after each op with the full variable names whose gradient that op just
        wrote (the data-parallel exchange launches a bucket once all its parameters are final, ddp.py)."""
        main = torch.cuda.current_stream()
        try:
            return self._backward(run, grad_outputs, need_input_grad, on_grads, grad_accumulate)
        finally:
            torch.cuda.set_stream(main)

    def _backward(self, run, grad_outputs, need_input_grad, on_grads, grad_accumulate):
        pacc = 1 if grad_accumulate else 0
        N = run.N
        if self.pre_backward is not None:
            self.pre_backward()
        lib = _lib.load()
        st = _lib.stream_ptr()
        spec = self.spec
        run.ensure_grad()
        written = {b.name: [] for b in spec.bufs}

        def mark(v):
            """Return accumulate flag for writing gradient view v and record it."""
            lst = written[v.buf.name]
            lo, hi = v.coff, v.coff + v.C
            for a, b in lst:
                if a <= lo and hi <= b:
                    return 1
                assert hi <= a or b <= lo, f"partial gradient overlap on {v.buf.name}"
            lst.append((lo, hi))
            return 0

        for v, g in zip(spec.outputs, grad_outputs):
            acc = mark(v)
            if isinstance(g, str) and g == IN_PLACE:
                assert acc == 0, "an in-place output gradient must be the view's only gradient"
                continue
            if g is None:
                g = torch.empty((N, v.H, v.W, v.C), device=run.device, dtype=torch.float32)
                _lib.check(lib.tde_fill(g.numel(), ptr(g), 0.0, st), "zero grad_out")
            g = g.contiguous()
            _lib.check(lib.tde_copy_view(N * v.H * v.W, v.C, ptr(g), v.C, 0, run.vptr(v, True), v.buf.cs, v.coff,
                                         acc, st), "grad_out")
        ws, dz = self._scratch(N)
        wsb = ws.numel() * 4
        iv = spec.input_view
        _lib.check(lib.tde_zero_bytes(run.absmax.numel() * 4, ptr(run.absmax), st), "zero dz bounds")
        side = self.wgrad_stream if self._production() else None
        if side is SERIAL:
            side = torch.cuda.current_stream()
        if side is not None:
            self._wg_N = N
            self._wg_pending, self._wg_issued = [], []
        conv_rank = {}
        for j, o in enumerate(spec.ops):
            if isinstance(o, ConvBN):
                conv_rank[j] = len(conv_rank)
        tl = self.timeline
        for i in range(len(spec.ops) - 1, -1, -1):
            op = spec.ops[i]
            if tl is not None and i + 1 < len(spec.ops):
                tl.mark(self.prefix, "B", spec.ops[i + 1])
            if self.timer is not None:
                self.timer.tag = getattr(op, "layer", type(op).__name__)
            src_needs = need_input_grad or op.src.buf is not spec.input
            if isinstance(op, ConvBN):
                use_side = side is not None and conv_rank[i] >= 1   # (the first layer: no data gradient)
                d = op.desc(N)
                self._use_split(d, i, N)
                # dz (the conv's output gradient) is the y view of a conv's descriptor, the x view of a deconv's
                if op.deconv:
                    d.x_absmax = run.absmax_ptr(i)
                else:
                    d.y_absmax = run.absmax_ptr(i)
                M = N * op.dst.H * op.dst.W
                sm = run.stats.get(i)
                if side is not None:
                    dz = self._dz_layer(N, i, M * op.K)
                if not op.bn:
                    # BN-free layer: dz = dy * relu'(y), bias gradient (fixed-order fp64 sums)
                    with self._span("bn_bwd"):
                        _lib.check(lib.tde_bias_relu_bwd(M, op.K, run.vptr(op.dst), op.dst.buf.cs, op.dst.coff,
                                                         run.vptr(op.dst, True), op.dst.buf.cs, op.dst.coff, 1, ptr(dz),
                                                         ptr(self.G(f"{op.layer}/biases")), pacc, run.absmax_ptr(i),
                                                         ptr(ws), wsb, st), op.layer + " bias_relu_bwd")
                elif self.bn_sync is not None:
                    # SyncBN backward: local (sum g, sum g*xhat) per row group (one launch writes the copy to be
                    # all-reduced and the local one) -> all-reduce -> dz from the global means in one launch; dbeta
                    # from the local sums, groups added in order (the gradient all-reduce averages it like every
                    # parameter)
                    G = run.groups
                    Mg = M // G
                    ls, gs = self._sums(i, op.K, 1, G), self._sums(i, op.K, 2, G)
                    beta = self.P(f"{op.layer}/BatchNorm/beta")
                    zi = run.z[i]
                    dy = run.vptr(op.dst, True)
                    _lib.check(lib.tde_bn_sums(M, op.K, G, ptr(zi), dy, op.dst.buf.cs, op.dst.coff, ptr(sm[0]),
                                               ptr(sm[1]), ptr(beta), 1, 1, ptr(gs), ptr(ls), ptr(ws), wsb, st),
                               op.layer + " bn sums")
                    self.bn_sync(gs)
                    _lib.check(lib.tde_bn_bwd_from_sums(M, op.K, G, Mg * self.bn_world, ptr(zi), ptr(sm[0]), ptr(sm[1]),
                                                        ptr(beta), dy, op.dst.buf.cs, op.dst.coff, ptr(gs), ptr(ls),
                                                        ptr(dz), ptr(self.G(f"{op.layer}/BatchNorm/beta")), pacc, 1,
                                                        run.absmax_ptr(i), st), op.layer + " syncbn bwd")
                else:
                    with self._span("bn_bwd"):
                        _lib.check(lib.tde_bn_bwd(M, op.K, run.groups, ptr(run.z[i]), ptr(sm[0]), ptr(sm[1]),
                                                  ptr(self.P(f"{op.layer}/BatchNorm/beta")), run.vptr(op.dst, True),
                                                  op.dst.buf.cs, op.dst.coff, ptr(dz),
                                                  ptr(self.G(f"{op.layer}/BatchNorm/beta")), pacc, 1,
                                                  run.absmax_ptr(i), ptr(ws), wsb, st), op.layer + " bn_bwd")
                w, gw = self.P(f"{op.layer}/weights"), self.G(f"{op.layer}/weights")
                fl = conv_flops(op, N)
                if use_side:
                    # this layer's filter gradient joins the deferred group; the group goes to the side stream
                    # behind one event recorded after the BN backward that completes it.  The data gradient is
                    # issued BEFORE the side stream waits on that event: under capture the graph executor keeps
                    # a node's first-added successor on the node's own HW queue, so the data-gradient chain
                    # stays on one queue and only the filter-gradient branch forks off it
                    wg = lib.tde_deconv2d_bwd_filter if op.deconv else lib.tde_conv2d_bwd_filter
                    a1, a2 = (ptr(dz), run.vptr(op.src)) if op.deconv else (run.vptr(op.src), ptr(dz))

                    def wgrad_call(wsp, wsb2, wg=wg, d=d, a1=a1, a2=a2, gw=gw, layer=op.layer, fl=fl, op=op):
                        with self._span("conv_wgrad", fl, conv_bytes(op, N)):
                            _lib.check(wg(ctypes_ref(d), a1, a2, ptr(gw), pacc, wsp, wsb2, _lib.stream_ptr()),
                                       layer + " wgrad")
                    self._wg_pending.append((wgrad_call, [f"{self.prefix}/{n}" for n, _, _ in op.params]))
                    ev = torch.cuda.Event()
                    ev.record()
                    if src_needs:
                        acc = mark(op.src)
                        with self._span("conv_dgrad", fl, conv_bytes(op, N)):
                            if op.deconv:
                                _lib.check(lib.tde_deconv2d_bwd_data(ctypes_ref(d), ptr(dz), ptr(w),
                                                                     run.vptr(op.src, True), acc, ptr(ws), wsb, st),
                                           op.layer + " bwd data")
                            else:
                                _lib.check(lib.tde_conv2d_bwd_data(ctypes_ref(d), ptr(dz), ptr(w), run.vptr(op.src, True),
                                                                   acc, ptr(ws), wsb, st), op.layer + " bwd data")
                    self._flush_wgrad(ev)
                elif src_needs:
                    # data + filter gradient: one fused launch (tde_conv2d_bwd / tde_deconv2d_bwd)
                    acc = mark(op.src)
                    with self._span("conv_bwd", 2 * fl, 2 * conv_bytes(op, N)):
                        if op.deconv:
                            _lib.check(lib.tde_deconv2d_bwd(ctypes_ref(d), ptr(dz), run.vptr(op.src), ptr(w),
                                                            run.vptr(op.src, True), acc, ptr(gw), pacc, ptr(ws), wsb,
                                                            st), op.layer + " bwd")
                        else:
                            _lib.check(lib.tde_conv2d_bwd(ctypes_ref(d), run.vptr(op.src), ptr(dz), ptr(w),
                                                          run.vptr(op.src, True), acc, ptr(gw), pacc, ptr(ws), wsb,
                                                          st), op.layer + " bwd")
                else:
                    # first layer: no input gradient
                    wg = lib.tde_deconv2d_bwd_filter if op.deconv else lib.tde_conv2d_bwd_filter
                    a1, a2 = (ptr(dz), run.vptr(op.src)) if op.deconv else (run.vptr(op.src), ptr(dz))
                    with self._span("conv_wgrad", fl, conv_bytes(op, N)):
                        _lib.check(wg(ctypes_ref(d), a1, a2, ptr(gw), pacc, ptr(ws), wsb, st), op.layer + " wgrad")
                if side is not None:
                    # report the parameters of the filter gradients issued so far (a deferred one is reported
                    # once its group is on the side stream)
                    names, self._wg_issued = self._wg_issued, []
                    if not use_side:
                        names += [f"{self.prefix}/{n}" for n, _, _ in op.params]
                    if on_grads is not None and names:
                        on_grads(names)
                elif on_grads is not None:
                    on_grads([f"{self.prefix}/{n}" for n, _, _ in op.params])
            elif isinstance(op, Head):
                d = op.desc(N)
                acc = mark(op.src) if src_needs else 0
                hw, hgw, hgb = (ptr(self.P(f"{op.layer}/weights")), ptr(self.G(f"{op.layer}/weights")),
                                ptr(self.G(f"{op.layer}/biases")))
                if side is not None:
                    # the head's filter gradient joins the deferred group on the side stream (it reads x, y and
                    # dy, none of which the rest of backward rewrites); the data gradient stays on this stream
                    def head_wgrad_call(wsp, wsb2, d=d, x=run.vptr(op.src), y=run.vptr(op.dst),
                                        dy=run.vptr(op.dst, True), op=op, hw=hw, hgw=hgw, hgb=hgb):
                        _lib.check(lib.tde_head_bwd(ctypes_ref(d), x, hw, y, dy, None, 0, hgw, hgb, pacc, op.act,
                                                    op.scale, op.offset, wsp, wsb2, _lib.stream_ptr()),
                                   op.layer + " head wgrad")
                    self._wg_pending.append((head_wgrad_call, [f"{self.prefix}/{n}" for n, _, _ in op.params]))
                    ev = torch.cuda.Event()
                    ev.record()
                    if src_needs:
                        _lib.check(lib.tde_head_bwd(ctypes_ref(d), run.vptr(op.src), hw, run.vptr(op.dst),
                                                    run.vptr(op.dst, True), run.vptr(op.src, True), acc, None, None,
                                                    0, op.act, op.scale, op.offset, ptr(ws), wsb, st),
                                   op.layer + " head dgrad")
                    self._flush_wgrad(ev)
                    names, self._wg_issued = self._wg_issued, []
                    if on_grads is not None and names:
                        on_grads(names)
                    continue
                with self._span("head_bwd", 2 * conv_flops(op, N)):
                    _lib.check(lib.tde_head_bwd(ctypes_ref(d), run.vptr(op.src), hw,
                                                run.vptr(op.dst), run.vptr(op.dst, True),
                                                run.vptr(op.src, True) if src_needs else None, acc,
                                                hgw, hgb, pacc, op.act, op.scale, op.offset, ptr(ws), wsb, st),
                               op.layer + " bwd")
                if on_grads is not None:
                    on_grads([f"{self.prefix}/{n}" for n, _, _ in op.params])
            elif isinstance(op, Resize):
                s, t = op.src, op.dst
                acc = mark(s)
                fn = lib.tde_resize_nearest_bwd if op.kind == "nearest" else lib.tde_resize_bilinear_bwd
                with self._span("resize"):
                    _lib.check(fn(N, s.H, s.W, s.C, run.vptr(s, True), s.buf.cs, s.coff, acc, t.H, t.W,
                                  run.vptr(t, True), t.buf.cs, t.coff, st), op.kind + " bwd")
            elif isinstance(op, Copy):
                s, t = op.src, op.dst
                acc = mark(s)
                _lib.check(lib.tde_copy_view(N * s.H * s.W, s.C, run.vptr(t, True), t.buf.cs, t.coff,
                                             run.vptr(s, True), s.buf.cs, s.coff, acc, st), "copy bwd")
        if tl is not None and spec.ops:
            tl.mark(self.prefix, "B", spec.ops[0])
        if side is not None:
            self._flush_wgrad()
            names, self._wg_issued = self._wg_issued, []
            if on_grads is not None and names:
                on_grads(names)
            self.join_wgrad()
        if need_input_grad:
            return run.view_tensor(iv, grad=True)[..., :spec.cin]
        return None


def ctypes_ref(d):
    import ctypes
    return ctypes.byref(d)


class KernelTimer:
    """HIP-event spans on the current stream, summed per kernel family (used by bench.py on an
    instrumented eager step; never active inside a captured graph)."""

    def __init__(self):
        self.spans = []   # (family, start_event, end_event, flops, tag)
        self.tag = None   # set by the executor to the current layer name
        self.nbytes = {}  # family -> algorithmic bytes

    def span(self, family, flops=0.0, nbytes=0.0):
        self.nbytes[family] = self.nbytes.get(family, 0.0) + nbytes
        return _Span(self, family, flops)

    def totals(self):
        torch.cuda.synchronize()
        out = {}
        for fam, a, b, fl, _ in self.spans:
            t, f, n = out.get(fam, (0.0, 0.0, 0))
            out[fam] = (t + a.elapsed_time(b), f + fl, n + 1)
        return out   # family -> (ms, flops, launches)

    def by_tag(self):
        torch.cuda.synchronize()
        return [(fam, tag, a.elapsed_time(b), fl) for fam, a, b, fl, tag in self.spans]


class GraphTimer:
    """Conv-kernel spans of the PRODUCTION step as captured and replayed (bench.py's roofline): each conv entry
    call is preceded by tde_conv_span_arm with a fresh pair of device timestamp slots; the library launches a
    one-wave stamp kernel (100 MHz real-time counter) right before the call's first conv-family kernel and one right
    after its last (split-K reduce included, the BatchNorm launches of a fused conv + BN call excluded).  Captured,
    the stamps are nodes of the step's graphs; after a replay, end - begin per span is the time its kernels took
    where the graph ran them (filter gradients on their side stream, two networks on two streams).  Only the conv
    families are timed; every other span is a no-op, and nothing is recorded outside a capture."""

    graph = True
    FAMILIES = ("conv_fwd", "conv_bwd", "conv_dgrad", "conv_wgrad")
    TICK_MS = 1e-5        # s_memrealtime: 100 MHz

    def __init__(self, max_spans=2048):
        self.spans = []   # (family, span index, flops, tag)
        self.tag = None
        self.nbytes = {}
        self.stamps = torch.zeros((max_spans, 2), dtype=torch.int64, device="cuda")

    def span(self, family, flops=0.0, nbytes=0.0):
        if family not in self.FAMILIES or not torch.cuda.is_current_stream_capturing():
            return NO_SPAN
        if len(self.spans) >= self.stamps.shape[0]:
            raise _lib.TdeError("GraphTimer: more conv calls than max_spans")
        self.nbytes[family] = self.nbytes.get(family, 0.0) + nbytes
        return _GraphSpan(self, family, flops)

    def per_span_ms(self):
        """[(family, tag, ms, flops)] of the LAST replay (call after a replay and a synchronize)."""
        st = self.stamps.cpu()
        return [(fam, tag, float(st[k, 1] - st[k, 0]) * self.TICK_MS, fl) for fam, k, fl, tag in self.spans]

    def busy_ms(self):
        """Wall time of the last replay during which at least one conv span was open: the union of the spans'
        [begin, end] intervals over all the step's streams (the stamp counter is device-wide), so concurrent
        kernels on two or three streams are not counted twice."""
        st = self.stamps.cpu()
        iv = sorted((int(st[k, 0]), int(st[k, 1])) for _, k, _, _ in self.spans)
        tot, cur_a, cur_b = 0, None, None
        for a, b in iv:
            if cur_b is None or a > cur_b:
                if cur_b is not None:
                    tot += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        if cur_b is not None:
            tot += cur_b - cur_a
        return tot * self.TICK_MS

    def totals(self):
        """family -> (ms, flops, calls) of the last replay."""
        out = {}
        for fam, _, ms, fl in self.per_span_ms():
            t, f, n = out.get(fam, (0.0, 0.0, 0))
            out[fam] = (t + ms, f + fl, n + 1)
        return out


class StepTimeline:
    """Diagnostic step timeline (probe/step_timeline.py): under capture, a device stamp (tde_stamp, the 100 MHz
    real-time counter) is appended to the stream an op ran on right after the op's launches; after a replay, an op's
    time is its stamp minus the previous stamp on the same stream -- its kernels plus any cross-stream wait it began
    with.  The stamp kernels are extra graph nodes (about a microsecond each), so the replay is slower than the
    production step; the picture of which stream is busy with what, not the total, is the point."""

    TICK_US = 1e-2

    def __init__(self, max_marks=8192):
        self.stamps = torch.zeros(max_marks, dtype=torch.int64, device="cuda")
        self.marks = []       # (label, stream handle)

    def mark(self, prefix, phase, op_or_label):
        if not torch.cuda.is_current_stream_capturing():
            return
        if len(self.marks) >= self.stamps.numel():
            raise _lib.TdeError("StepTimeline: more marks than max_marks")
        name = op_or_label if isinstance(op_or_label, str) else getattr(op_or_label, "layer", type(op_or_label).__name__)
        if not isinstance(op_or_label, str) and getattr(op_or_label, "branch", 0):
            name += " [branch]"
        s = torch.cuda.current_stream()
        _lib.check(_lib.load().tde_stamp(ctypes.c_void_p(self.stamps.data_ptr() + 8 * len(self.marks)),
                                         ctypes.c_void_p(s.cuda_stream)), "stamp")
        self.marks.append((f"{phase} {prefix.split('/')[0]}:{name}", s.cuda_stream))

    def intervals(self):
        """[(label, stream, start_us, end_us)] of the last replay: per stream, marks in issue order."""
        st = self.stamps.cpu().tolist()
        last, out = {}, []
        for k, (label, sid) in enumerate(self.marks):
            t = st[k]
            if sid in last:
                out.append((label, sid, last[sid] * self.TICK_US, t * self.TICK_US))
            last[sid] = t
        return out


class _GraphSpan:
    def __init__(self, timer, family, flops):
        self.timer, self.family, self.flops = timer, family, flops

    def __enter__(self):
        self.k = len(self.timer.spans)
        base = self.timer.stamps.data_ptr() + 16 * self.k
        _lib.load().tde_conv_span_arm(ctypes.c_void_p(base), ctypes.c_void_p(base + 8))
        return self

    def __exit__(self, *exc):
        n = _lib.load().tde_conv_span_arm(None, None)
        if exc[0] is None:
            if n != 2:
                raise _lib.TdeError(f"conv span of {self.timer.tag}: {n} stamps launched, expected 2")
            self.timer.spans.append((self.family, self.k, self.flops, self.timer.tag))
        return False


class _Span:
    def __init__(self, timer, family, flops):
        self.timer, self.family, self.flops = timer, family, flops

    def __enter__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)
        self.a.record()
        return self

    def __exit__(self, *exc):
        self.b.record()
        self.timer.spans.append((self.family, self.a, self.b, self.flops, self.timer.tag))
        return False


class _NoSpan:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


NO_SPAN = _NoSpan()


def conv_bytes(op, N):
    """Algorithmic HBM bytes of one conv / deconv call in any of its three modes: each reads two of
    {x, w, y} and writes the third, once (fp32)."""
    if not isinstance(op, ConvBN):
        return 0.0
    if op.deconv:
        x = N * op.dst.H * op.dst.W * op.K
        y = N * op.src.H * op.src.W * op.src.creal
    else:
        x = N * op.src.H * op.src.W * op.src.creal
        y = N * op.OH * op.OW * op.K
    return 4.0 * (x + y + op.k * op.k * op.src.creal * op.K)


def conv_flops(op, N):
    """Algorithmic MACs*2 of one conv / deconv layer (all taps of the dense conv)."""
    if isinstance(op, ConvBN):
        if op.deconv:
            return 2.0 * N * op.src.H * op.src.W * op.K * op.k * op.k * op.src.creal
        return 2.0 * N * op.OH * op.OW * op.K * op.k * op.k * op.src.creal
    if isinstance(op, Head):
        return 2.0 * N * op.src.H * op.src.W * op.K * op.k * op.k * op.src.creal
    return 0.0
