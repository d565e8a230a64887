#!/usr/bin/env python3
"""Training-throughput benchmark (BASELINE.json metric: training image-pairs/sec at 256x192).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2|config3|config4|config5]
                    [--batch B] [--no-graph] [--no-cpu-baseline] [--no-secondary]
For N > 1 launch with `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`:
one process per GPU, per-GPU batch fixed (weak scaling), gradients averaged with bucketed RCCL
all-reduces overlapped with backward.

A step = one pass of the hot path over one synthetic batch already resident in HBM: network
forward(s), fused loss head (values + gradients), backward(s), Adam.  The default workload is the
metric's pair path, config 4 (train_depth_then_cam_lr.py:123-154,211-355: 2x disp_net + 2x 4-scale
depth_net, photometric warp loss, per-GPU batch 8 = the 8-GPU shard of global batch 64): 1 unit =
1 image pair.  Config 2 (BASELINE configs[1], single images) and config 3 (pairs, batch 32) are
timed after it on rank 0 at N = 1 as the `secondary` object; config 5 is selectable.  The step is
recorded into hipGraphs and replayed.

Prints ONE JSON line on rank 0 with
  roofline    : the MFMA implicit-GEMM conv family (fwd + dgrad + wgrad): algorithmic FLOPs of the
                step's convs / their summed HIP-event time, measured live on an instrumented step on
                the stream the kernels run on, against the dense fp16 MFMA peak / 3 (fp16x3 math);
                mfma_busy / traffic from the committed rocprofv3 PMC summary of the same workload;
  cpu_baseline: the oracle's PyTorch-CPU fp32 restatement of the same step ("port": TF-1 cannot
                run here), timed on a bounded sample on this host's cores, rank 0 at N = 1 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3        # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
BF16_MFMA_PEAK = 2500.0              # MI355X_MICROARCH.md: Peak BF16 MFMA, dense (~2.5 PF)
METRIC = "training image-pairs/sec at 256x192, 1/2/4/8 MI355X; depth L1 vs ref"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- synthetic inputs
def texture(rng, B, H, W):
    """Smooth random texture: sum of 8 random sinusoids + 0.02 N(0,1), clipped to +-0.5."""
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    out = np.zeros((B, H, W, 3), np.float32)
    for b in range(B):
        for c in range(3):
            for _ in range(8):
                fx, fy = rng.uniform(0.02, 0.25, 2)
                out[b, :, :, c] += rng.uniform(0.05, 0.15) * np.sin(fx * xx + fy * yy + rng.uniform(0, 6.28))
    out += 0.02 * rng.standard_normal(out.shape).astype(np.float32)
    return torch.from_numpy(np.clip(out, -0.5, 0.5))


def intrinsics(B, H, W):
    """Normalized (fx,fy,cx,cy) = (0.89,1.19,0.5,0.5) x (W,H), per-scale / 2^s (Demon_Data_loader.py:25-39)."""
    K = np.zeros((B, 4, 3, 3), np.float32)
    for s in range(4):
        f = 2.0 ** s
        K[:, s] = [[0.89 * W / f, 0, 0.5 * W / f], [0, 1.19 * H / f, 0.5 * H / f], [0, 0, 1]]
    return torch.from_numpy(K)


def small_pose(rng, B):
    t = rng.standard_normal((B, 3))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    ax = rng.standard_normal((B, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    return torch.tensor(np.concatenate([t, ax * rng.uniform(0.02, 0.2, (B, 1))], 1), dtype=torch.float32)


def rodrigues_np(v):
    """pose vector (t, angle-axis r) -> 4x4 (data prep for the configs whose pose is a given matrix)."""
    T = np.tile(np.eye(4, dtype=np.float32), (v.shape[0], 1, 1))
    for b, (tx, ty, tz, rx, ry, rz) in enumerate(v.numpy().astype(np.float64)):
        th = np.sqrt(rx * rx + ry * ry + rz * rz)
        a = np.array([rx, ry, rz]) / th
        Kx = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        T[b, :3, :3] = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
        T[b, :3, 3] = [tx, ty, tz]
    return torch.from_numpy(T)


WORKLOADS = {
    # name: (H, W, default per-GPU batch, train GFLOP per unit, description)
    "config2": (192, 256, 8, 20.05, "config2: train_depth_only.py path -- nets_optflow_depth.disp_net fwd + "
                                    "smooth/depth-L1 loss head + bwd + Adam (BASELINE configs[1])"),
    "config3": (192, 256, 32, 30.22, "config3: train_optflow_combine.py path -- nets_depth joint depth+flow net + "
                                     "GT-warp wmask, depth/flow warps, flow L1, smooth + Adam"),
    "config4": (192, 256, 8, 89.37, "config4: train_depth_then_cam_lr.py path -- 2x disp_net + 2x 4-scale "
                                    "depth_net, photometric/exp/consistency/cam loss + Adam (per-GPU shard of 64)"),
    "config5": (480, 640, 2, 125.9, "config5: refine_depth.py path -- disp_net at 640x480 + warp/depth/smooth "
                                    "loss + Adam (per-GPU shard of 16)"),
}


def make_trainer(name, N):
    from tf_depth_estimation_amd import train
    H, W = WORKLOADS[name][:2]
    cls = dict(config2=train.DepthOnlyTrainer, config3=train.OptflowCombineTrainer,
               config4=train.DepthThenCamTrainer, config5=train.RefineTrainer)[name]
    return cls(N, H, W)


def make_batch(name, N, seed):
    H, W = WORKLOADS[name][:2]
    rng = np.random.default_rng(seed)
    if name == "config2":
        x = torch.tensor(rng.uniform(-0.5, 0.5, (N, H, W, 3)), dtype=torch.float32)
        lab = torch.tensor(rng.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32)
        return (x, lab)
    if name == "config3":
        il, ir = texture(rng, N, H, W), texture(rng, N, H, W)
        lab = torch.tensor(rng.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32)
        T = rodrigues_np(small_pose(rng, N) * torch.tensor([0.1, 0.1, 0.1, 1, 1, 1]))
        return (il, ir, lab, intrinsics(N, H, W), T)
    if name == "config4":
        il, ir = texture(rng, N, H, W), texture(rng, N, H, W)
        lab = rng.uniform(0.1, 2.0, (N, H, W, 1)).astype(np.float32)
        lab[rng.uniform(size=lab.shape) < 0.05] = np.nan
        return (il, ir, torch.from_numpy(lab), intrinsics(N, H, W), small_pose(rng, N))
    x1, x2 = texture(rng, N, H, W), texture(rng, N, H, W)
    gt = torch.tensor(rng.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32)
    T = rodrigues_np(small_pose(rng, N) * torch.tensor([0.1, 0.1, 0.1, 1, 1, 1]))
    return (x1, x2, gt, intrinsics(N, H, W), T)


# ---------------------------------------------------------------- depth L1 vs the reference (CPU leg)
def depth_l1_vs_ref(name, N, seed=7):
    """The metric's second half ("depth L1 vs ref"): the workload's network forward on the
    GPU (public API, fresh Glorot variables, training-mode BN, the benched conv math) against the float64
    oracle restatement of the same graph on identical inputs and weights.  Per output: mean |gpu - ref|
    and max|gpu - ref| / max|ref| (north-star bar 1e-4).  Runs in the CPU-baseline leg (rank 0, N = 1)."""
    from oracle import nets as ON
    from tf_depth_estimation_amd import _api, variables
    from tf_depth_estimation_amd import nets_depth, nets_optflow_depth, nets_optflow_depth_pairtest
    H, W = WORKLOADS[name][:2]
    rng = np.random.default_rng(seed)

    def oracle_params(chunk):
        P = ON.Params(dtype=torch.float64)
        for v in chunk.names():
            P.vars[v] = chunk.view(v).detach().double().cpu().clone()
        return P

    def img(C):
        return torch.tensor(rng.uniform(-0.5, 0.5, (N, H, W, C)), dtype=torch.float32)

    pairs = []   # (label, gpu outputs, oracle outputs)
    with torch.no_grad(), variables.variable_scope("bench_ref_check"):
        if name == "config3":
            x = img(6)
            outs, ep = nets_depth.disp_net(x.cuda(), is_training=True)
            ref = ON.disp_net_depthflow(oracle_params(ep["program"].chunk), x.double(), True,
                                        scope="bench_ref_check/depth_net")
            pairs += [(f"{'disp' if i < 4 else 'flow'}{i % 4 + 1}", o, r) for i, (o, r) in enumerate(zip(outs, ref))]
        else:
            x = img(3)
            outs, ep = nets_optflow_depth.disp_net(x.cuda(), is_training=True)
            ref = ON.disp_net(oracle_params(ep["program"].chunk), x.double(), True, scope="bench_ref_check/depth_net")
            pairs += [(f"disp{i + 1}", o, r) for i, (o, r) in enumerate(zip(outs, ref))]
            if name == "config4":
                x6 = img(6)
                d, pose, m, ep = nets_optflow_depth_pairtest.depth_net(x6.cuda(), is_training=True)
                rd, rp, rm = ON.depth_net(oracle_params(ep["program"].chunk), x6.double(), True,
                                          scope="bench_ref_check/depth_cam_net", levels=4)
                pairs += [(f"pair_disp{i + 1}", o, r) for i, (o, r) in enumerate(zip(d, rd))]
                pairs += [("pose", pose, rp)]
    _api.clear_programs()
    res = {}
    for lab, o, r in pairs:
        g = o.detach().double().cpu()
        r = r.detach().double()
        res[lab] = {"mean_abs": float((g - r).abs().mean()), "max_rel": float((g - r).abs().max() / r.abs().max())}
    worst = max(v["max_rel"] for v in res.values())
    return {"outputs": res, "worst_max_rel": worst, "tol": 1e-4, "pass": worst <= 1e-4,
            "sample": f"{N} x {W}x{H} synthetic input(s), fresh Glorot weights, training-mode BN, "
                      "float64 oracle restatement (oracle/nets.py)"}


# ---------------------------------------------------------------- CPU baseline (oracle restatement)
def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Host threads for the CPU leg: every core this process may run on (sched_getaffinity), capped by an
    explicit OMP_NUM_THREADS (the GPU box sets it to its per-GPU CPU share; os.cpu_count() there reports the
    whole machine, and oversubscribing it would understate the CPU path)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        cap = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        cap = 0
    return min(n, cap) if cap > 0 else n


def cpu_baseline(name, N, budget_s=12.0):
    from oracle import losses as OL
    from oracle import nets as ON
    threads = cpu_threads()
    torch.set_num_threads(threads)
    H, W = WORKLOADS[name][:2]
    batch = make_batch(name, N, 0)
    Ps = ON.Params(dtype=torch.float32)
    Pp = ON.Params(dtype=torch.float32)
    opt = OL.AdamTF(lr=2e-4)

    def step():
        for P in (Ps, Pp):
            for v in P.vars.values():
                v.grad = None
        if name == "config2":
            x, lab = batch
            loss, _ = OL.loss_depth_only(ON.disp_net(Ps, x, True, scope="model/depth_net"), lab)
        elif name == "config3":
            il, ir, lab, K, T = batch
            outs = ON.disp_net_depthflow(Ps, torch.cat([il, ir], -1), True, scope="model/depth_net")
            loss, _ = OL.loss_optflow_combine(outs, il, ir, lab, K, T)
        elif name == "config4":
            il, ir, lab, K, gt = batch
            dsl = ON.disp_net(Ps, il, True, scope="model_singledepth/depth_net")
            dsr = ON.disp_net(Ps, ir, True, scope="model_singledepth/depth_net")
            dpl, pr, ml = ON.depth_net(Pp, torch.cat([il, ir], -1), True, scope="model_pairdepth/depth_cam_net")
            dpr, pl, mr = ON.depth_net(Pp, torch.cat([ir, il], -1), True, scope="model_pairdepth/depth_cam_net")
            loss, _ = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, il, ir, lab, K, gt)
        else:
            x1, x2, gt, K, T = batch
            loss, _ = OL.loss_refine(ON.disp_net(Ps, x1, True, scope="model/depth_net"), x1, x2, gt, T, K)
        loss.backward()
        params = dict(Ps.vars, **Pp.vars)
        opt.step(params, {k: v.grad for k, v in params.items()})

    step()  # warm-up (creates variables)
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 20:
            break
    return dict(value=round(N * n / el, 3), unit="image-pairs/s", cores=threads, kind="port",
                cpu_model=cpu_model(), host_cpus=os.cpu_count(),
                sample=f"{n} {name} training steps x {N} samples at {W}x{H}, PyTorch-CPU fp32 restatement "
                       f"(oracle/), {el:.1f}s wall")


def build_trainer(args, name, N, world, rank):
    """Trainer for `name` with the benched options (exchange, overlaps); returns (trainer, options dict)."""
    from tf_depth_estimation_amd import train
    tr = make_trainer(name, N)
    tr.set_batch(*[t.cuda() for t in make_batch(name, N, seed=1000 + rank)])
    if world > 1 or args.exchange == "on":
        # (--exchange on at N = 1: a world-1 RCCL group, so the N > 1 exchange path is timed on one GPU)
        if args.ddp == "overlap":
            tr.enable_ddp(world, bucket_mb=args.bucket_mb, mode=args.exchange_mode)
        else:
            tr.grad_sync = train.MultiAllReduce(tr.chunks, world)
    if args.sync_bn:
        tr.enable_sync_bn(world)
    net_overlap = (args.net_overlap == "on" and args.adam_overlap == "off" and
                   len(tr.programs()) > 1 and not (args.deferred_adam == "on" and world == 1))
    wg_progs = []
    if args.wgrad_overlap == "on":
        only = None
        if args.wgrad_progs == "auto":
            # config 4 with the net overlap: only depth_net (the second stream's network, the longer chain) moves
            # its filter gradients to a side stream; disp_net's stay fused on the compute stream, which then
            # carries a chain as long as depth_net's (measured: 980 vs 910 pairs/s with both moved, 866 with
            # only disp_net's)
            if net_overlap and getattr(tr, "ov_net", None) == "pair" and not os.environ.get("TDE_WGRAD_PROGS"):
                only = ["pair"]
        elif args.wgrad_progs != "all":
            only = args.wgrad_progs.split(",")
        tr.enable_wgrad_overlap(only=only)
        wg_progs = [n for n in ("prog", "single", "pair")
                    if getattr(getattr(tr, n, None), "wgrad_stream", None) is not None]
    if args.adam_overlap != "off" and world == 1:
        tr.enable_adam_overlap(args.adam_bucket_mb, on_wgrad_stream=args.adam_overlap == "wgrad")
    deferred = args.deferred_adam == "on" and world == 1 and args.adam_overlap == "off" and not args.sync_bn
    if deferred:
        tr.enable_deferred_adam()
    if net_overlap:
        tr.enable_net_overlap()
    return tr, dict(deferred=deferred, net_overlap=net_overlap, wgrad_progs=wg_progs)


def instrumented_step(tr):
    """One eager step with per-family HIP-event spans on the stream the kernels run on (outside the timed
    region; the instrumented step runs its programs serially on one stream)."""
    from tf_depth_estimation_amd.program import KernelTimer
    progs = tr.programs()
    tr.step_eager()
    tr.flush()       # no update in flight during the instrumented step
    timer = KernelTimer()
    for p in progs:
        p.timer = timer
    tr.step_eager()
    for p in progs:
        p.timer = None
    tr.flush()
    return timer.totals(), timer.nbytes


def graph_timed_conv(tr, replays=7):
    """The conv family as the TIMED schedule runs it: the production step captured with a GraphTimer (an event-
    record node before and after each conv entry call's kernels, program.GraphTimer), replayed `replays` times on
    the trainer's streams; per family the median over replays of the summed span times.  Then the graphs are
    dropped (the timed region captures its own, without event nodes)."""
    from tf_depth_estimation_amd.program import GraphTimer
    progs = tr.programs()
    timer = GraphTimer()
    for p in progs:
        p.timer = timer
    try:
        tr.capture()
    finally:
        for p in progs:
            p.timer = None
    per, spans, busy = [], None, []
    for _ in range(replays):
        tr.step()
        torch.cuda.synchronize()
        per.append(timer.totals())
        busy.append(timer.busy_ms())
        spans = timer.per_span_ms()
    tr.flush()
    tr.release_graphs()
    torch.cuda.synchronize()
    out = {}
    for fam in per[0]:
        ms = sorted(p[fam][0] for p in per)
        out[fam] = (ms[len(ms) // 2], per[0][fam][1], per[0][fam][2])
    busy.sort()
    return out, spans, busy[len(busy) // 2]


def timed_steps(tr, steps, warmup, world, rank, use_graph):
    if use_graph:
        tr.capture()
    for _ in range(warmup):
        tr.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.step()
        if i % 50 == 49:
            log(f"[bench] rank {rank} step {i + 1}/{steps}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    return el


def conv_family(fam):
    conv = [fam[k] for k in ("conv_fwd", "conv_bwd", "conv_dgrad", "conv_wgrad") if k in fam]
    return sum(c[0] for c in conv), sum(c[1] for c in conv), sum(c[2] for c in conv)


# Environment variables that change what a step computes or how it is scheduled for DIAGNOSTICS (timing
# experiments, serial replays): a bench line is never taken with one set.  (The work-skipping switches exist only in
# a -DTDE_TIMING_DIAG build of libtde.so; the shipped library ignores them, and bench refuses them anyway.)
DIAG_ENV = ("TDE_SKIP_CONV_LE", "TDE_SKIP_CONV_GT", "TDE_SKIP_WHAT", "TDE_SKIP_WGRAD", "TDE_HWG_DIAG",
            "TDE_DBG_PHASE")


def env_knobs():
    """Every TDE_* tuning variable set in the environment (reported in the line); refuse the diagnostic ones."""
    set_ = {k: v for k, v in os.environ.items() if k.startswith("TDE_")}
    bad = sorted(k for k in set_ if k in DIAG_ENV)
    if bad:
        raise SystemExit(f"bench.py: diagnostic environment variables set ({', '.join(bad)}): refusing to measure")
    return set_


def main():
    # the ONE JSON line goes to the original stdout; everything native libraries print there (RCCL's version banner at
    # communicator creation, for one) is sent to stderr instead, so stdout holds nothing but the line
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="config4", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: the workload's)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--math", default="fp16x3", choices=["fp32", "bf16x3", "bf16x6", "bf16x6r", "fp16x3"],
                    help="conv arithmetic (include/tde.h tde_set_conv_math): exact fp32 MFMA, bf16x3 split "
                         "precision, the fp32-accurate 3-way bf16 split (LDS-staged / register-split) or the "
                         "fp32-accurate scaled 2-way fp16 split (3 fp16 MFMAs per product; the default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph-spans", default="", help="write the per-call conv spans of the graph timing (JSON)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary workloads (configs 2, 3 and 5 timed after the headline at N = 1)")
    ap.add_argument("--bucket-mb", type=float, default=256.0,
                    help="gradient all-reduce bucket size (N > 1): 256 = one bucket per network; smaller buckets fork "
                         "the comm branch mid-backward, measured slower on one GPU (ddp.py)")
    ap.add_argument("--adam-overlap", default="off", choices=["off", "side", "wgrad"],
                    help="N = 1: run each gradient bucket's Adam as soon as backward finalises it, on its own side "
                         "stream or on the filter-gradient stream")
    ap.add_argument("--adam-bucket-mb", type=float, default=16.0)
    ap.add_argument("--deferred-adam", default="off", choices=["on", "off"],
                    help="N = 1: run each step's Adam at the start of the next step on a side stream, overlapped with "
                         "its forward (per-bucket waits; bit-identical updates; every timed step still runs one "
                         "full Adam).  Measured: config 2 1.1 %% slower, config 4 equal (HBM contention)")
    ap.add_argument("--wgrad-overlap", default="on", choices=["on", "off"],
                    help="filter gradients on a side stream, off backward's data-gradient chain (a parallel graph "
                         "branch; bit-identical results)")
    ap.add_argument("--wgrad-progs", default="auto",
                    help="programs whose filter gradients go to a side stream: auto (config 4 with the net overlap: "
                         "'pair'; else all), all, or a comma list of single,pair,prog (TDE_WGRAD_PROGS when unset)")
    ap.add_argument("--net-overlap", default="on", choices=["on", "off"],
                    help="config 4: depth_net's calls on a second stream beside disp_net's (independent "
                         "programs; one graph per piece, replayed with stream waits; bit-identical results). "
                         "Measured config 4 605 -> 665 samples/s")
    ap.add_argument("--sync-bn", action="store_true",
                    help="BatchNorm over the global batch (one RCCL all-reduce of every row group's sums per BN layer "
                         "and direction, on a communicator of its own, captured into the step's graphs)")
    ap.add_argument("--ddp", default="overlap", choices=["overlap", "after"],
                    help="N > 1: bucketed all-reduce overlapped with backward, or one all-reduce after it")
    ap.add_argument("--exchange", default="auto", choices=["auto", "on"],
                    help="gradient exchange: auto = with N > 1; on = also at N = 1 over a world-1 RCCL group (times the "
                         "multi-GPU code path on one GPU)")
    ap.add_argument("--exchange-mode", default="segments", choices=["graph", "segments"],
                    help="bucket all-reduces (direct RCCL, one communicator per network) issued by the host between "
                         "graph segments cut at each bucket launch point, on the reporting network's own stream, each "
                         "network's Adam inline after its exchange (segments, the default since round 6), or captured "
                         "into the step's graphs on per-network comm branches (graph; refused with the net overlap at "
                         "N > 1, see ddp.py)")
    args = ap.parse_args()
    knobs = env_knobs()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1 or args.sync_bn or args.exchange == "on":
        # (--sync-bn at N = 1: a world-1 RCCL group, so the SyncBN step -- sums kernels and the captured
        # all-reduce nodes -- runs as it does at N > 1)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))

    from tf_depth_estimation_amd import _api, _lib, variables

    H, W, Nd, gflop_unit, desc = WORKLOADS[args.workload]
    N = args.batch or Nd
    _lib.check(_lib.load().tde_set_conv_math(_lib.CONV_MATH[args.math]), "conv math")
    tr, opts = build_trainer(args, args.workload, N, world, rank)
    fam, fam_bytes = instrumented_step(tr)
    use_graph = not args.no_graph
    # roofline: measured on the captured production schedule the timed region replays (N = 1); the instrumented
    # eager step (conv and BN as separate calls, one stream) stays in the line as kernel_breakdown_ms
    gfam = None
    gbusy = None
    if use_graph and world == 1:
        gfam, gspans, gbusy = graph_timed_conv(tr)
        if args.graph_spans:
            with open(args.graph_spans, "w") as fh:
                json.dump([{"family": f, "layer": t, "ms": round(ms, 5), "gflop": fl / 1e9} for f, t, ms, fl in gspans],
                          fh, indent=0)
        span_sum_ms, conv_flops, conv_launches = conv_family(gfam)
        conv_ms = gbusy
    else:
        conv_ms, conv_flops, conv_launches = conv_family(fam)
    el = timed_steps(tr, args.steps, args.warmup, world, rank, use_graph)
    loss = tr.total_loss()
    tr.flush()       # deferred Adam: apply the last step's owed update (outside the timed region)

    if rank == 0:
        if args.math != "fp32":
            # 3 or 6 bf16/fp16 MFMAs per fp32 product: the algorithmic fp32 FLOPs are counted once and priced
            # against the dense bf16/fp16 MFMA peak (the same rate) divided by the MFMAs per product (the rate
            # at which this arithmetic can retire fp32 products), so frac = fraction of the matrix pipe doing
            # useful work
            per = 6 if args.math in ("bf16x6", "bf16x6r") else 3
            ins = "v_mfma_f32_16x16x32_f16" if args.math == "fp16x3" else "v_mfma_f32_16x16x32_bf16"
            kernel_name = (f"igemmx_kernel<{_lib.CONV_MATH[args.math]},...> + halo_conv_kernel + hwh_kernel (conv "
                           f"fwd+dgrad+wgrad, {args.math}: {per} x {ins} per fp32 product)")
            peak = round(BF16_MFMA_PEAK / per, 1)
            peak_note = f"dense bf16/fp16 MFMA peak {BF16_MFMA_PEAK} TFLOP/s / {per} MFMAs per fp32 product"
        else:
            kernel_name, peak = "igemmx_kernel<0,...> (conv fwd+dgrad+wgrad, fp32 MFMA 16x16x4)", FP32_MFMA_PEAK_TFLOPS
            peak_note = "dense fp32 MFMA peak"
        value = world * N * args.steps / el
        achieved = conv_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
        dtype = {"fp16x3": "fp16x3", "fp32": "f32"}.get(args.math, args.math)
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "image-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "dtype_note": ("fp32 tensors end to end; the convolutions split each fp32 operand into scaled fp16 hi/lo "
                           "parts and run 3 fp16 MFMAs per product with fp32 accumulation (fp32-class accuracy, "
                           "DESIGN.md §2); BatchNorm, heads, loss head and Adam compute in fp32 (fp64 reductions)"
                           if args.math == "fp16x3" else f"conv math {args.math}"),
            "data": "synthetic (SURVEY.md §8d shapes/distributions); random-init Glorot weights",
            "config": {"workload": desc, "global_batch": world * N, "per_gpu_batch": N, "resolution": f"{W}x{H}",
                       "parallelism": f"dp{world}", "hip_graph": use_graph,
                       # captured graphs of the step and the cuts the exchange forces between them (graph mode: the
                       # bucket all-reduces are graph nodes, so 0; segments mode: one cut per bucket launch point)
                       "graph_segment_cuts": tr.segment_cuts() if use_graph else None,
                       "grad_exchange": (None if world == 1 and args.exchange != "on" else
                                         f"{args.ddp}, {args.bucket_mb} MB buckets, {args.exchange_mode}"),
                       "batch_norm": "sync (global batch)" if args.sync_bn else "per-replica batch",
                       "wgrad_overlap": args.wgrad_overlap == "on", "wgrad_progs": opts.get("wgrad_progs"),
                       "adam_overlap": args.adam_overlap if world == 1 else "off",
                       "deferred_adam": opts["deferred"],
                       "net_overlap": opts["net_overlap"],
                       "unit_note": "1 unit = 1 training sample: an image pair (configs 3/4); configs 2/5 train on "
                                    "one image of it"},
            "roofline": {"bound": "mfma", "kernel": kernel_name, "math": args.math,
                         "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "peak_note": peak_note, "traffic": None,
                         "frac_of_dense_fp16_peak": round(achieved / BF16_MFMA_PEAK, 4),
                         "frac_of_dense_fp16_peak_note": ("achieved fp32-equivalent conv TFLOP/s / the 2.5 PF dense fp16 MFMA "
                                                         "peak the north star names (each fp32 product costs 3 fp16 "
                                                         "MFMAs in fp16x3, so 1/3 is this arithmetic's ceiling)"),
                         "timing": ("conv-busy wall time of the captured production step: a one-wave stamp kernel "
                                    "(device real-time counter) before and after every conv entry call's kernels "
                                    "inside the graphs the timed region replays (less the stamps), the union of the "
                                    "stamped intervals over the step's 2-3 concurrent streams, median of 7 replays"
                                    if gfam is not None else
                                    "HIP events around each conv call of an instrumented eager step on one stream"),
                         "sum_of_call_spans_ms": round(span_sum_ms, 4) if gfam is not None else None,
                         "sum_of_call_spans_note": ("per-call spans added up: calls running concurrently on "
                                                    "different streams each count in full (their kernels share the "
                                                    "CUs), so this exceeds the busy time" if gfam is not None
                                                    else None),
                         "family_ms_per_step": ({k: round(v[0], 4) for k, v in sorted(gfam.items())}
                                                if gfam is not None else None),
                         "flops_per_step": conv_flops, "conv_ms_per_step": round(conv_ms, 4),
                         "conv_calls_per_step": conv_launches,
                         "survey_flops_per_step": gflop_unit * 1e9 * N},
            "kernel_breakdown_ms": {k: round(v[0], 4) for k, v in sorted(fam.items())},
            "env_knobs": knobs,
            "final_loss": loss,
        }
        tr_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}_{args.math}_b{N}.json")
        if os.path.exists(tr_path):
            # HBM bytes and MFMA-pipe busy from rocprofv3 --pmc passes of this workload (scripts/pmc_step.sh, a
            # separate profiled run: counters cannot be read inside this timed process)
            with open(tr_path) as fh:
                pm = json.load(fh)
            conv_t = pm["families"].get("conv", {})
            rf = out["roofline"]
            rf["traffic"] = conv_t.get("hbm_bytes_per_step")
            rf["traffic_unit"] = "bytes per step, conv family (igemm + halo + split-K reduce)"
            rf["traffic_algorithmic"] = sum(v for k, v in fam_bytes.items() if k.startswith("conv_"))
            if "mfma_busy" in conv_t:
                rf["mfma_busy"] = round(conv_t["mfma_busy"], 4)
                rf["mfma_busy_note"] = ("SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs) over the conv "
                                        "family's dispatches (includes the 2 redundant fp16 products of fp16x3 and "
                                        "tile padding)")
            if conv_t.get("hbm_bytes_per_step") and conv_ms > 0:
                rf["hbm_gbs"] = round(conv_t["hbm_bytes_per_step"] / (conv_ms * 1e-3) / 1e9, 1)
                rf["hbm_gbs_note"] = ("PMC conv-family bytes per step / the conv family's busy time per step measured "
                                      "here (the roofline's timing): no clock assumption")
            rf["traffic_source"] = os.path.relpath(tr_path, ROOT)
            rf["traffic_label"] = pm.get("label")
        if world == 1 and not args.no_secondary:
            sec = {}
            for name in ("config2", "config3", "config5"):
                if name == args.workload:
                    continue
                log(f"[bench] secondary workload {name} ...")
                del tr
                _api.clear_programs()
                variables.get_store().reset()
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
                tr, o2 = build_trainer(args, name, WORKLOADS[name][2], 1, 0)
                f2, _ = instrumented_step(tr)
                cm, cf, _ = conv_family(f2)
                e2 = timed_steps(tr, args.steps, args.warmup, 1, 0, use_graph)
                n2 = WORKLOADS[name][2]
                sec[name] = {"value": round(n2 * args.steps / e2, 3), "unit": "image-pairs/s",
                             "ms_per_step": round(e2 / args.steps * 1e3, 4), "per_gpu_batch": n2,
                             "workload": WORKLOADS[name][4],
                             "conv_tflops": round(cf / (cm * 1e-3) / 1e12, 3) if cm > 0 else None}
            out["secondary"] = sec
        if world == 1 and not args.no_cpu_baseline:
            log("[bench] timing CPU baseline ...")
            out["cpu_baseline"] = cpu_baseline(args.workload, N)
            log("[bench] depth L1 vs the float64 reference restatement ...")
            out["depth_l1_vs_ref"] = depth_l1_vs_ref(args.workload, N)
        print(json.dumps(out), file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
