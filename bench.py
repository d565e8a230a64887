#!/usr/bin/env python3
"""Training-throughput benchmark (BASELINE.json metric: training image-pairs/sec at 256x192).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2] [--no-graph]
                    [--no-cpu-baseline]
For N > 1 launch with `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`:
one process per GPU, per-GPU batch fixed (weak scaling), gradients averaged with one RCCL
all-reduce of the flat gradient buffer per step.

A step = one pass of the hot path over one synthetic batch already resident in HBM: disp_net
forward, fused loss head (value + gradient), backward, Adam (BASELINE config 2, train_depth_only.py,
per-GPU batch 8 = configs[1]).  The step is recorded once into a hipGraph and replayed.

Prints ONE JSON line on rank 0 (contract in the task brief), with
  roofline    : the MFMA implicit-GEMM conv family (fwd + dgrad + wgrad), algorithmic FLOPs of the
                step's convs / their summed HIP-event time, measured live on an instrumented step,
                against the fp32 MFMA dense peak (157.3 TFLOP/s, MI355X_MICROARCH.md);
  cpu_baseline: the oracle's PyTorch-CPU fp32 restatement of the same step ("port": TF-1 cannot
                run here), timed on a bounded sample on this host's cores.
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
TRAIN_GFLOP_PER_IMAGE = 20.05        # disp_net train GFLOP/image at 256x192


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_batch(N, H, W, seed):
    """images U(-0.5,0.5), label disparity U(0.25,4)."""
    g = np.random.default_rng(seed)
    x = torch.tensor(g.uniform(-0.5, 0.5, (N, H, W, 3)), dtype=torch.float32)
    lab = torch.tensor(g.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32)
    return x, lab


def cpu_baseline(N, H, W, budget_s=12.0):
    """Oracle restatement (PyTorch-CPU fp32) of the same config-2 step, bounded sample."""
    from oracle import losses as OL
    from oracle import nets as ON
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    x, lab = synthetic_batch(N, H, W, 0)
    P = ON.Params(dtype=torch.float32)
    opt = OL.AdamTF(lr=2e-4)

    def step():
        for v in P.vars.values():
            v.grad = None
        ref = ON.disp_net(P, x, True, scope="model/depth_net")
        loss, _ = OL.loss_depth_only(ref, lab)
        loss.backward()
        opt.step(P.vars, {k: v.grad for k, v in P.vars.items()})

    step()  # warm-up (creates variables)
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 20:
            break
    return dict(value=round(N * n / el, 3), unit="image-pairs/s", cores=threads, kind="port",
                sample=f"{n} config-2 training steps x {N} images at {W}x{H}, PyTorch-CPU fp32 restatement "
                       f"(oracle/), {el:.1f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8, help="per-GPU batch (config 4: 64 global / 8 GPUs)")
    ap.add_argument("--workload", default="config2", choices=["config2"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    from tf_depth_estimation_amd import train
    from tf_depth_estimation_amd.program import KernelTimer

    H, W, N = 192, 256, args.batch
    tr = train.DepthOnlyTrainer(N, H, W)
    x, lab = synthetic_batch(N, H, W, seed=rank)
    tr.set_batch(x.cuda(), lab.cuda())
    if world > 1:
        tr.grad_sync = train.MultiAllReduce(tr.chunks, world)

    # instrumented eager step: per-family HIP-event times for the roofline
    tr.step_eager()
    timer = KernelTimer()
    tr.prog.timer = timer
    tr.step_eager()
    tr.prog.timer = None
    fam = timer.totals()
    conv = [fam[k] for k in ("conv_fwd", "conv_dgrad", "conv_wgrad") if k in fam]
    conv_ms = sum(c[0] for c in conv)
    conv_flops = sum(c[1] for c in conv)
    conv_launches = sum(c[2] for c in conv)

    use_graph = not args.no_graph
    if use_graph:
        tr.capture()
    for _ in range(args.warmup):
        tr.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        tr.step()
        if i % 50 == 49:
            log(f"[bench] rank {rank} step {i + 1}/{args.steps}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    loss = tr.total_loss()

    if rank == 0:
        value = world * N * args.steps / el
        achieved = conv_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
        out = {
            "metric": "training image-pairs/sec at 256x192, 1/2/4/8 MI355X; depth L1 vs ref",
            "value": round(value, 3),
            "unit": "image-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (SURVEY.md §8d: images U(-0.5,0.5), label disparity U(0.25,4)); random-init "
                    "Glorot weights",
            "config": {"workload": "config2: train_depth_only.py path -- nets_optflow_depth.disp_net fwd + "
                                   "smooth/depth-L1 loss head + bwd + Adam (configs[1])",
                       "global_batch": world * N, "per_gpu_batch": N, "resolution": f"{W}x{H}",
                       "parallelism": f"dp{world}", "hip_graph": use_graph,
                       "unit_note": "config 2 trains on the left image of each loaded pair: 1 pair = 1 sample"},
            "roofline": {"bound": "mfma", "kernel": "igemm_kernel (conv fwd+dgrad+wgrad, fp32 MFMA 16x16x4)",
                         "achieved": round(achieved, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                         "flops_per_step": conv_flops, "conv_ms_per_step": round(conv_ms, 4),
                         "launches_per_step": conv_launches,
                         "survey_flops_per_step": TRAIN_GFLOP_PER_IMAGE * 1e9 * N},
            "kernel_breakdown_ms": {k: round(v[0], 4) for k, v in sorted(fam.items())},
            "final_loss": loss,
        }
        if world == 1 and not args.no_cpu_baseline:
            log("[bench] timing CPU baseline ...")
            out["cpu_baseline"] = cpu_baseline(N, H, W)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
