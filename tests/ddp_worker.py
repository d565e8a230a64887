"""Rank program for tests/test_ddp.py, launched on CPU as
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ... tests/ddp_worker.py CASE
with the gloo backend.  It drives tf_depth_estimation_amd.ddp.GradSync with the real disp_net
schedule (reverse op order = the order NetProgram.backward reports finished parameters) on a CPU
ParamChunk, and asserts on every rank; a non-zero exit fails the test.

  mean        : rank-dependent gradients -> every rank ends with the exact fp32 mean, buckets fire
                during the schedule (not all at the end), each exactly once.
  uses2       : shared-variable net reported twice per step (config 4): nothing fires on pass 1.
  oracle_step : one data-parallel config-2 step: each rank takes its shard of the global batch,
                computes the oracle gradient, writes it op by op with hooks; after the exchange and
                the oracle Adam, parameters are bit-identical across ranks and equal to Adam applied
                to the mean of the gathered per-rank gradients.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tf_depth_estimation_amd import _netlib, ddp  # noqa: E402
from tf_depth_estimation_amd.variables import ParamChunk  # noqa: E402

PREFIX = "model/depth_net"


def build(H=128, W=128):
    spec = _netlib.disp_net_spec(H, W, 3)
    specs, bn = spec.param_specs()
    chunk = ParamChunk([(f"{PREFIX}/{n}", s, i) for n, s, i in specs], [(f"{PREFIX}/{n}", c) for n, c in bn],
                       device="cpu", seed=1)
    return spec, chunk


def schedule(spec):
    """Parameter names in the order backward reports them (one list per op)."""
    return [[f"{PREFIX}/{n}" for n, _, _ in op.params] for op in reversed(spec.ops) if op.params]


def gather(t):
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return out


def case_mean(rank, world):
    spec, chunk = build()
    gs = ddp.GradSync([chunk], world, bucket_mb=1.0)
    assert len(gs.buckets) > 4
    g = torch.Generator().manual_seed(100 + rank)
    src = torch.randn(chunk.numel, generator=g)
    expect = sum(torch.randn(chunk.numel, generator=torch.Generator().manual_seed(100 + r)) for r in range(world))
    expect = expect * (1.0 / world)
    # padding elements between parameters belong to buckets too
    pad = torch.ones(chunk.numel, dtype=torch.bool)
    for n in chunk.names():
        o = chunk.offsets[n]
        pad[o:o + chunk.grad_view(n).numel()] = False
    chunk.grad[pad] = src[pad]
    gs.begin_step()
    hook = gs.hook(chunk)
    fired_at = []
    sched = schedule(spec)
    for i, names in enumerate(sched):
        for n in names:
            o = chunk.offsets[n]
            chunk.grad[o:o + chunk.grad_view(n).numel()] = src[o:o + chunk.grad_view(n).numel()]
        before = len(gs.log)
        hook(names)
        fired_at += [i] * (len(gs.log) - before)
    gs.finish()
    assert all(b.launched for b in gs.buckets)
    assert sum(len(x) for x in gs.log) == len(chunk.names()), "every parameter exchanged exactly once"
    assert fired_at and fired_at[0] < len(sched) // 2, f"first bucket only at op {fired_at[0]}/{len(sched)}"
    assert torch.equal(chunk.grad, expect), "mean mismatch (padding included)"
    allg = gather(chunk.grad)
    assert all(torch.equal(allg[0], x) for x in allg)


def case_uses2(rank, world):
    spec, chunk = build()
    gs = ddp.GradSync([chunk], world, bucket_mb=1.0, uses={id(chunk): 2})
    gs.begin_step()
    hook = gs.hook(chunk)
    chunk.grad.fill_(float(rank + 1))
    for names in schedule(spec):
        hook(names)
    assert not gs.log, "a bucket fired before the second backward pass"
    for names in schedule(spec):
        hook(names)
    assert all(b.launched for b in gs.buckets) and not gs.leftovers()
    gs.finish()
    assert torch.all(chunk.grad == sum(range(1, world + 1)) / world)


def case_oracle_step(rank, world):
    from oracle import losses as OL
    from oracle import nets as ON
    spec, chunk = build()
    N_global, H, W = 2 * world, 128, 128
    rng = np.random.default_rng(7)
    imgs = torch.tensor(rng.uniform(-0.5, 0.5, size=(N_global, H, W, 3)), dtype=torch.float32)
    labs = torch.tensor(rng.uniform(0.25, 4.0, size=(N_global, H, W, 1)), dtype=torch.float32)
    lo, hi = rank * N_global // world, (rank + 1) * N_global // world
    P = ON.Params(dtype=torch.float64)
    for n in chunk.names():
        P.vars[n] = chunk.view(n).detach().double().clone().requires_grad_(True)
    out = ON.disp_net(P, imgs[lo:hi].double(), True, scope=PREFIX)
    loss, _ = OL.loss_depth_only(out, labs[lo:hi].double())
    loss.backward()
    mine = torch.zeros_like(chunk.grad)
    for n in chunk.names():
        o = chunk.offsets[n]
        mine[o:o + chunk.grad_view(n).numel()] = P.vars[n].grad.reshape(-1).float()
    gs = ddp.GradSync([chunk], world, bucket_mb=2.0)
    gs.begin_step()
    chunk.grad.zero_()
    hook = gs.hook(chunk)
    for names in schedule(spec):
        for n in names:
            chunk.grad_view(n).add_(mine[chunk.offsets[n]:chunk.offsets[n] + chunk.grad_view(n).numel()]
                                    .view_as(chunk.grad_view(n)))
        hook(names)
    gs.finish()
    allg = gather(mine)
    expect = allg[0].clone()
    for x in allg[1:]:
        expect += x
    expect *= 1.0 / world
    assert torch.equal(chunk.grad, expect), "exchanged gradient != mean of per-rank gradients"
    opt = OL.AdamTF(lr=2e-4)
    with torch.no_grad():
        params = {n: chunk.view(n).double().clone() for n in chunk.names()}
        opt.step(params, {n: chunk.grad_view(n).double() for n in chunk.names()})
        flat = torch.cat([params[n].reshape(-1) for n in chunk.names()])
    allp = gather(flat)
    assert all(torch.equal(allp[0], x) for x in allp), "replicas diverged after the update"


def main():
    case = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    try:
        {"mean": case_mean, "uses2": case_uses2, "oracle_step": case_oracle_step}[case](rank, world)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if rank == 0:
        print(f"ddp_worker {case} ok (world {world})")


if __name__ == "__main__":
    main()
