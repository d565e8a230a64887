"""Training steps for the BASELINE configs, as static schedules of libtde.so calls.

A step is fwd + fused loss head (forward and its hand-derived gradient in one pass) + bwd + Adam,
all on one HIP stream over buffers allocated once, so `Trainer.capture()` can record the whole step
into a hipGraph (torch.cuda.CUDAGraph) and replay it with zero host work per step.

  DepthOnlyTrainer   config 2 -- train_depth_only.py:108-219 (disp_net, smooth + depth L1, Adam)
"""
import torch

from . import _api, _lib, _netlib, variables
from ._lib import ptr
from .program import NetRun

W_CONFIG2 = dict(smooth=1.0, depth=1.0)     # train_depth_only.py:33-37


class Adam:
    """tf.train.AdamOptimizer(lr, beta1) over one ParamChunk (flat buffers)."""

    def __init__(self, chunk, lr=2e-4, beta1=0.9, beta2=0.999, eps=1e-8):
        self.chunk, self.lr, self.b1, self.b2, self.eps = chunk, lr, beta1, beta2, eps
        self.t = torch.zeros(1, device="cuda", dtype=torch.float32)

    def step(self):
        lib, st = _lib.load(), _lib.stream_ptr()
        c = self.chunk
        _lib.check(lib.tde_adam_step_begin(ptr(self.t), st), "adam step")
        _lib.check(lib.tde_adam_update(c.numel, ptr(c.flat), ptr(c.grad), ptr(c.adam_m), ptr(c.adam_v), ptr(self.t),
                                       self.lr, self.b1, self.b2, self.eps, st), "adam")


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
    """Common capture/replay machinery.  A step is phase_compute (zero grads, fwd, loss, bwd),
    the optional gradient exchange, then phase_update (Adam).  Without an exchange the whole step is
    one hipGraph; with one, compute and update are two graphs and the RCCL all-reduce runs between
    their replays on the same stream."""

    graphs = None
    grad_sync = None

    def step_eager(self):
        self.phase_compute()
        if self.grad_sync is not None:
            self.grad_sync()
        self.phase_update()

    def capture(self, warmup=2):
        """Warm up on a side stream (allocates every lazily created buffer), then record."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_eager()
        torch.cuda.current_stream().wait_stream(s)
        if self.grad_sync is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.phase_compute()
                self.phase_update()
            self.graphs = [g]
        else:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                self.phase_compute()
            with torch.cuda.graph(g2):
                self.phase_update()
            self.graphs = [g1, g2]
        return self.graphs

    def step(self):
        if self.graphs is None:
            self.step_eager()
        elif len(self.graphs) == 1:
            self.graphs[0].replay()
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
        self.run = NetRun(self.prog, batch)
        self.opt = Adam(self.chunk, lr, beta1)
        dev = "cuda"
        self.images = torch.zeros(batch, H, W, 3, device=dev, dtype=torch.float32)
        self.label = torch.ones(batch, H, W, 1, device=dev, dtype=torch.float32)
        self.label_pyr = [self.label] + [torch.empty(batch, H >> s, W >> s, 1, device=dev, dtype=torch.float32) for s in (1, 2, 3)]
        outs = self.prog.spec.outputs
        self.d_out = [torch.empty(batch, v.H, v.W, v.C, device=dev, dtype=torch.float32) for v in outs]
        self.loss = torch.zeros(1, dtype=torch.float64, device=dev)
        self.parts = torch.zeros(2, dtype=torch.float64, device=dev)   # [depth, smooth]

    def set_batch(self, images, label):
        self.images.copy_(images)
        self.label.copy_(label)

    def phase_update(self):
        self.opt.step()

    def phase_compute(self):
        lib, st = _lib.load(), _lib.stream_ptr()
        c = self.chunk
        _lib.check(lib.tde_zero_bytes(c.numel * 4, ptr(c.grad), st), "zero grad")
        _lib.check(lib.tde_zero_bytes(16, ptr(self.parts), st), "zero loss")
        for g in self.d_out:
            _lib.check(lib.tde_zero_bytes(g.numel() * 4, ptr(g), st), "zero dout")
        outs = self.prog.forward(self.run, self.images, True)
        N, H, W = self.N, self.H, self.W
        for s in (1, 2, 3):
            _lib.check(lib.tde_resize_area_fwd(N, H, W, 1, ptr(self.label), H >> s, W >> s, ptr(self.label_pyr[s]),
                                               st), "label pyramid")
        p_depth = ctypes_double_ptr(self.parts, 0)
        p_smooth = ctypes_double_ptr(self.parts, 1)
        for s in range(4):
            pred, g = outs[s], self.d_out[s]
            h, w = pred.shape[1], pred.shape[2]
            _lib.check(lib.tde_loss_smooth2(N, h, w, ptr(pred), 1, 0, 0, self.w["smooth"] / 2 ** s, p_smooth, ptr(g),
                                            1, 0, st), "smooth")
            _lib.check(lib.tde_loss_l1(N, h, w, ptr(pred), 1, 0, ptr(self.label_pyr[s]), 0, self.w["depth"] / 2 ** s,
                                       p_depth, ptr(g), 1, 0, st), "depth l1")
        self.prog.backward(self.run, self.d_out)

    def total_loss(self):
        return float(self.parts.sum().item())

    def outputs(self):
        return [self.run.view_tensor(v) for v in self.prog.spec.outputs]


def ctypes_double_ptr(t, idx):
    import ctypes
    return ctypes.c_void_p(t.data_ptr() + 8 * idx)
