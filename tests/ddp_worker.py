"""Rank program for tests/test_ddp.py, launched on CPU as
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ... tests/ddp_worker.py CASE
with the gloo backend.  It drives tf_depth_estimation_amd.ddp.GradSync with the real disp_net
schedule (reverse op order = the order NetProgram.backward reports finished parameters) on a CPU
ParamChunk, and asserts on every rank; a non-zero exit fails the test.

  mean        : rank-dependent gradients -> every rank ends with the exact fp32 mean, buckets fire
                during the schedule (not all at the end), each exactly once.
  uses2       : shared-variable net reported twice per step (config 4): nothing fires on pass 1.
  two_programs: config 4 with the net overlap: disp_net's and depth_net's chunks in ONE GradSync, one backward
                call each (twin batching, uses 1), their reports interleaved as two streams would issue them,
                with the pre_launch / side_streams callbacks of Trainer.enable_ddp; each bucket fires once
                during its own program's schedule, the launch callbacks see the reporting chunk, and both
                chunks end with the exact mean.
  syncbn      : the SyncBN protocol of Trainer.enable_sync_bn / NetProgram (per-layer fp64 (sum z, sum z^2) and, in
                backward, (sum g, sum g*xhat) all-reduced with SUM; statistics and coefficients from the global
                sums over M x world rows; dbeta from the LOCAL sum, averaged by the gradient exchange), restated
                with the formulas of bn.hip's stats_from_sums / bn_bwd_apply_kernel: every rank's normalised
                output, dz, dbeta and moving averages equal whole-batch BatchNorm + ReLU (oracle tf_ops.batch_norm
                and its fp64 autograd) on the concatenated batch, the reference's one-device semantics
                (train_depth_then_cam_lr.py:130-136).  The kernels themselves run on the GPU in
                tests/test_gpu_ddp_world2.py (c2_syncbn).
  order       : the issue order of a step's collectives is the program order on every rank, whatever the timing
                (VERDICT r05 item 2): config 4's two chunks in one GradSync (the default segments mode), each rank
                sleeping a different random time before each report and inside each collective; every rank records
                the bucket order it issued, the orders are gathered and must be identical, and the exchanged
                gradients are the exact mean (a mismatched order would pair different buckets).
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


def case_two_programs(rank, world):
    spec_s, chunk_s = build()
    spec_p = _netlib.depth_net_spec(128, 128, 6, levels=4)
    specs, bn = spec_p.param_specs()
    pre_p = "model/depth_cam_net"
    chunk_p = ParamChunk([(f"{pre_p}/{n}", s, i) for n, s, i in specs], [(f"{pre_p}/{n}", c) for n, c in bn],
                         device="cpu", seed=2)
    seen = []
    gs = ddp.GradSync([chunk_s, chunk_p], world, bucket_mb=1.0, pre_launch=lambda c: seen.append(("pre", id(c))),
                      side_streams=lambda c: (seen.append(("side", id(c))), ())[1])
    gs.begin_step()
    hooks = {id(chunk_s): gs.hook(chunk_s), id(chunk_p): gs.hook(chunk_p)}
    chunk_s.grad.fill_(float(rank + 1))
    chunk_p.grad.fill_(float(10 * (rank + 1)))
    sched_s = schedule(spec_s)
    sched_p = [[f"{pre_p}/{n}" for n, _, _ in op.params] for op in reversed(spec_p.ops) if op.params]
    # interleave: depth_net's backward (the second stream) and disp_net's alternate op by op
    order = []
    for i in range(max(len(sched_s), len(sched_p))):
        if i < len(sched_p):
            order.append((chunk_p, sched_p[i]))
        if i < len(sched_s):
            order.append((chunk_s, sched_s[i]))
    fired = {id(chunk_s): 0, id(chunk_p): 0}
    for ch, names in order:
        before = len(gs.log)
        hooks[id(ch)](names)
        new = gs.log[before:]
        for nm in new:                  # every bucket that fired now belongs to the reporting chunk
            assert all(n.startswith(pre_p if ch is chunk_p else PREFIX + "/") for n in nm), (nm[:2], id(ch))
        fired[id(ch)] += len(new)
    assert fired[id(chunk_s)] > 0 and fired[id(chunk_p)] > 0, fired
    assert all(b.launched for b in gs.buckets) and not gs.leftovers(), "a bucket never reached its last report"
    assert all(kind == "side" for kind, _ in seen), "eager launches use side_streams, never pre_launch"
    assert {c for _, c in seen} == {id(chunk_s), id(chunk_p)}
    gs.finish()
    n = sum(range(1, world + 1)) / world
    assert torch.all(chunk_s.grad == n) and torch.all(chunk_p.grad == 10 * n)


def case_order(rank, world):
    import random
    import time
    spec_s, chunk_s = build()
    spec_p = _netlib.depth_net_spec(128, 128, 6, levels=4)
    specs, bn = spec_p.param_specs()
    pre_p = "model/depth_cam_net"
    chunk_p = ParamChunk([(f"{pre_p}/{n}", s, i) for n, s, i in specs], [(f"{pre_p}/{n}", c) for n, c in bn],
                         device="cpu", seed=2)
    gs = ddp.GradSync([chunk_s, chunk_p], world, bucket_mb=2.0)
    assert gs.mode == "segments"
    rnd = random.Random(1000 + rank)
    issued = []
    real = gs.launch

    def delayed_launch(buckets, streams=()):
        time.sleep(rnd.uniform(0, 0.004) * (rank + 1))
        issued.extend((b.chunk is chunk_p, b.lo, b.hi) for b in buckets)
        real(buckets, streams)
    gs.launch = delayed_launch
    for step in range(2):
        gs.begin_step()
        chunk_s.grad.fill_(float(rank + 1 + step))
        chunk_p.grad.fill_(float(10 * (rank + 1) + step))
        # the replay order of config 4's pieces: depth_net's chain (second stream) is issued before disp_net's
        for ch, sched in ((chunk_p, [[f"{pre_p}/{n}" for n, _, _ in op.params] for op in reversed(spec_p.ops)
                                      if op.params]),
                          (chunk_s, schedule(spec_s))):
            hook = gs.hook(ch)
            for names in sched:
                time.sleep(rnd.uniform(0, 0.0005))
                hook(names)
        gs.finish()
        n = sum(range(1, world + 1)) / world
        assert torch.all(chunk_s.grad == n + step) and torch.all(chunk_p.grad == 10 * n + step)
    orders = [None] * world
    dist.all_gather_object(orders, issued)
    assert len(issued) == 2 * len(gs.buckets)
    assert all(o == orders[0] for o in orders), "ranks issued their collectives in different orders"


def case_syncbn(rank, world):
    from oracle import tf_ops as T
    N, Hh, Ww, C = 3, 5, 7, 12           # per-rank shard: 105 rows x 12 channels
    eps, decay = 1e-3, 0.99
    g = torch.Generator().manual_seed(5)
    z_all = torch.randn(world * N, Hh, Ww, C, generator=g, dtype=torch.float64) * 2.0 + 0.3
    beta = torch.randn(C, generator=g, dtype=torch.float64) * 0.2
    dy_all = torch.randn(world * N, Hh, Ww, C, generator=g, dtype=torch.float64)
    mm0, mv0 = torch.randn(C, generator=g, dtype=torch.float64) * 0.1, torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    sl = slice(rank * N, (rank + 1) * N)
    z, dy_g = z_all[sl], dy_all[sl]
    M, Mt = N * Hh * Ww, world * N * Hh * Ww
    # ---- forward: local sums -> all-reduce (the Trainer's bn_sync) -> global statistics
    zf = z.reshape(-1, C)
    sums = torch.cat([zf.sum(0), (zf * zf).sum(0)])
    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    mean = sums[:C] / Mt
    var = (sums[C:] / Mt - mean * mean).clamp_min(0)
    invstd = 1.0 / torch.sqrt(var + eps)
    mm = mm0 - (mm0 - mean) * (1 - decay)
    mv = mv0 - (mv0 - var * Mt / (Mt - 1)) * (1 - decay)
    xh = (zf - mean) * invstd
    y = torch.relu(xh + beta).reshape(z.shape)
    # ---- reference: whole-batch BN + ReLU on one device (loss = mean over the global batch of <y, dy>)
    zr = z_all.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    st = T.BNState(C)
    st.moving_mean, st.moving_variance = mm0.clone(), mv0.clone()
    yr = torch.relu(T.batch_norm(zr, br, st, True, decay, eps))
    (yr * dy_all).sum().div(world * N).backward()
    assert torch.allclose(y, yr.detach()[sl], rtol=1e-12, atol=1e-12), "SyncBN forward != whole-batch BN"
    assert torch.allclose(mm, st.moving_mean, rtol=1e-12, atol=1e-14)
    assert torch.allclose(mv, st.moving_variance, rtol=1e-12, atol=1e-14)
    # ---- backward: this rank's loss is the mean over ITS shard, so its output gradient is world x the global one
    dyl = (dy_g / N).reshape(-1, C)
    gl = torch.where(xh + beta > 0, dyl, torch.zeros_like(dyl))
    lsum = torch.cat([gl.sum(0), (gl * xh).sum(0)])
    gsum = lsum.clone()
    dist.all_reduce(gsum, op=dist.ReduceOp.SUM)
    mg, mgx = gsum[:C] / Mt, gsum[C:] / Mt
    dz = invstd * (gl - mg - xh * mgx)
    dbeta = lsum[:C].clone()
    dist.all_reduce(dbeta, op=dist.ReduceOp.SUM)   # the gradient exchange: sum ...
    dbeta /= world                                  # ... and 1/world
    # d(global loss)/dz = d(local loss)/dz / world on this rank's rows
    assert torch.allclose(dz / world, zr.grad[sl].reshape(-1, C), rtol=1e-10, atol=1e-14), "SyncBN dz"
    # the exchanged dbeta (mean over ranks of the local sums) is d(global loss)/dbeta
    assert torch.allclose(dbeta, br.grad, rtol=1e-10, atol=1e-14), "SyncBN dbeta"


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
        {"mean": case_mean, "uses2": case_uses2, "two_programs": case_two_programs,
         "oracle_step": case_oracle_step, "syncbn": case_syncbn,
         "order": case_order}[case](rank, world)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if rank == 0:
        print(f"ddp_worker {case} ok (world {world})")


if __name__ == "__main__":
    main()
