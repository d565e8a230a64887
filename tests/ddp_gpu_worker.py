"""Rank program for tests/test_gpu_ddp_world2.py: TWO data-parallel ranks sharing the one GPU of the box (cuda:0),
launched as
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ... tests/ddp_gpu_worker.py CASE MODE
with the gloo backend (one card cannot host two RCCL ranks; gloo all-reduces the same device tensors through the
host).  Every rank runs the real GPU step -- kernels, the bucketed exchange on its comm stream, and with MODE=graph
the segmented piece capture whose replay interleaves graph segments with the bucket all-reduces -- and asserts; a
non-zero exit fails the test.  The global batch is 2 x B (rank r takes rows [rB, (r+1)B)).

  c4_local : config 4 (train_depth_then_cam_lr.py:123-154,211-355; twin batching with row-grouped BN, depth_net on
             the second stream, filter gradients on their side streams, deterministic warp-loss mode), BatchNorm
             over each replica's shard (the default).  After one step: the exchanged gradient equals
             the mean of the two ranks' local gradients (the same trainer without the exchange) bit for bit, lies
             within the oracle bars of the mean of the float64 oracle's per-shard gradients, and after Adam both
             replicas hold bit-identical parameters and moments.
  c2_syncbn: config 2 (train_depth_only.py) with SyncBN (Trainer.enable_sync_bn: per-layer fp64 sums all-reduced,
             every BN over the rows of BOTH ranks) and the overlapped exchange, eager: each rank's disparities equal
             the float64 oracle's whole-batch (2B) forward on its rows (1e-4), the mean of the rank losses equals the
             oracle's whole-batch loss (1e-5), and the exchanged gradient is the whole-batch gradient within the
             oracle bars -- the reference's single-device semantics at the global batch
             (train_depth_then_cam_lr.py:130-136: one BatchNorm batch per call).
  c4_syncbn: config 4 with twin batching and SyncBN: every row group (left images / right images, (L,R) pairs /
             (R,L) pairs) normalised over its rows on BOTH ranks, the groups' sums in one all-reduce per layer; each
             rank's outputs and poses equal the float64 oracle's four calls on the whole 2B batch (1e-4), the mean of
             the rank losses its loss terms (1e-5; consistency 1e-4), the exchanged gradient the whole-batch gradient
             within the oracle bars.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

B, H, W = 2, 64, 96


def gather(t):
    """All ranks' copies of a device tensor (gloo: through the host)."""
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return out


def c4_trainer(rank, ddp, mode):
    from test_gpu_trainers import intrinsics, small_pose, texture
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)          # identical initial variables on every rank
    _api.clear_programs()
    G = 2 * B
    il, ir = texture(G, H, W, 11), texture(G, H, W, 12)
    lab = torch.tensor(np.random.default_rng(13).uniform(0.1, 2.0, (G, H, W, 1)), dtype=torch.float32)
    K, gt = intrinsics(G, H, W), small_pose(G, 14)
    sl = slice(rank * B, (rank + 1) * B)
    tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
    tr.set_batch(il[sl].cuda(), ir[sl].cuda(), lab[sl].cuda(), K[sl].cuda(), gt[sl].cuda())
    tr.enable_wgrad_overlap(only=["pair"])
    if ddp:
        gs = tr.enable_ddp(dist.get_world_size(), bucket_mb=4.0)
        assert len(gs.buckets) > 4
    tr.enable_net_overlap()
    if mode == "graph":
        tr.capture(warmup=1)
        if ddp:
            nseg = sum(len(segs) for w, segs in tr.ov_seq if segs is not None)
            assert nseg > len([w for w, s in tr.ov_seq if s is not None]), "backward pieces were not cut"
    return tr, (il[sl], ir[sl], lab[sl], K[sl], gt[sl])


def case_c4_local(rank, world, mode):
    from oracle import losses as OL
    from oracle import nets as ON
    from test_gpu_nets import GRAD_FACTOR, check_grads_global, oracle_params_from
    from tf_depth_estimation_amd import _lib
    # local gradient of this rank's shard: the same trainer without the exchange (warm-up / capture steps update
    # the parameters, so both trainers are compared on the step they run from identical states: the first step
    # after construction, eagerly, for the local reference; the exchanged trainer's first step after its capture
    # is checked against parameters read before that step)
    ref, data = c4_trainer(rank, False, "eager")
    P64 = [oracle_params_from(c, "", torch.float64) for c in ref.chunks]
    P32 = [oracle_params_from(c, "", torch.float32) for c in ref.chunks]
    ref.phase_compute()
    torch.cuda.synchronize()
    local = [c.grad.clone() for c in ref.chunks]
    del ref
    tr, _ = c4_trainer(rank, True, mode)
    # the capture's warm-up ran steps: restart from the initial variables (same values on both ranks) so that the
    # checked step sees the parameters the local reference saw
    start = [c.flat.clone() for c in tr.chunks]
    for c, p in zip(tr.chunks, P64):
        for n in c.names():
            c.view(n).copy_(p.vars[n].detach().float().cuda())
        for bn_name in c.bn_offsets:
            m, v = c.moving(bn_name)
            m.copy_(p.bn[bn_name].moving_mean.float().cuda())
            v.copy_(p.bn[bn_name].moving_variance.float().cuda())
        c.adam_m.zero_()
        c.adam_v.zero_()
    for o in tr.opt.opts:
        o.t.zero_()
    del start
    tr.step()
    torch.cuda.synchronize()
    for c, g in zip(tr.chunks, local):
        al = gather(g)
        mean = (al[0] + al[1]) * (1.0 / world)
        assert torch.equal(c.grad, mean), "exchanged gradient != mean of the ranks' local gradients"
    # oracle: mean of the float64 per-shard gradients (BN over each shard, as the replicas compute)
    il, ir, lab, K, gt = data
    grads = {}
    for key, Ps in ((torch.float64, P64), (torch.float32, P32)):
        dt = key
        Pss, Ppp = Ps
        x = {"il": il.to(dt), "ir": ir.to(dt)}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        total, _ = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.to(dt),
                                             K.to(dt), gt.to(dt))
        total.backward()
        g = {}
        for P in Ps:
            for n, v in P.vars.items():
                loc = v.grad.detach().to(torch.float64)
                al = gather(loc.contiguous())
                g[n] = (al[0] + al[1]) / world
        grads[key] = g
    gpu = {}
    for c in tr.chunks:
        gpu.update({n: c.grad_view(n) for n in c.names()})
    e_gpu, e_cpu = check_grads_global(gpu, grads[torch.float64], grads[torch.float32],
                                      GRAD_FACTOR[_lib.load().tde_get_conv_math()])
    # replicas: bit-identical parameters and Adam moments after the update
    for c in tr.chunks:
        for t in (c.flat, c.adam_m, c.adam_v):
            al = gather(t)
            assert torch.equal(al[0], al[1]), "replicas diverged after the update"
    # a few more steps (replay keeps the exchange in step): replicas stay identical
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    for c in tr.chunks:
        al = gather(c.flat)
        assert torch.equal(al[0], al[1]), "replicas diverged over later steps"
    if rank == 0:
        print(f"c4_local {mode}: exchanged gradient vs fp64 oracle {e_gpu:.2e} (fp32 oracle {e_cpu:.2e})")


def case_c2_syncbn(rank, world, mode):
    from oracle import losses as OL
    from oracle import nets as ON
    from test_gpu_nets import GRAD_FACTOR, check_grads_global, oracle_params_from, rel_err
    from tf_depth_estimation_amd import _api, _lib, train, variables
    assert mode == "eager", "SyncBN all-reduces inside forward/backward: eager only"
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    G = 2 * B
    g = np.random.default_rng(21)
    x = torch.tensor(g.uniform(-0.5, 0.5, (G, H, W, 3)), dtype=torch.float32)
    lab = torch.tensor(g.uniform(0.25, 4.0, (G, H, W, 1)), dtype=torch.float32)
    sl = slice(rank * B, (rank + 1) * B)
    tr = train.DepthOnlyTrainer(B, H, W)
    tr.set_batch(x[sl].cuda(), lab[sl].cuda())
    tr.enable_sync_bn(world)
    tr.enable_ddp(world, bucket_mb=1.0)
    Ps = {dt: oracle_params_from(tr.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    tr.phase_compute()          # forward (SyncBN), loss, backward (SyncBN) with the bucketed exchange
    tr.grad_sync.finish()
    torch.cuda.synchronize()
    outs = [t.detach().cpu() for t in tr.outputs()]
    loss = torch.tensor([tr.total_loss()], dtype=torch.float64)
    al = gather(loss)
    mean_loss = (al[0].item() + al[1].item()) / world
    grads = {}
    for dt, P in Ps.items():
        d = ON.disp_net(P, x.to(dt), True, scope="model/depth_net")      # the WHOLE batch on one device
        lr, _ = OL.loss_depth_only(d, lab.to(dt))
        if dt == torch.float64:
            for i, (o, r) in enumerate(zip(outs, d)):
                e = rel_err(o, r[sl])
                assert e <= 1e-4, f"rank {rank} disp{i + 1}: SyncBN output vs whole-batch BN rel err {e:.2e}"
            assert abs(mean_loss - lr.item()) <= 1e-5 * abs(lr.item()), (mean_loss, lr.item())
        lr.backward()
        grads[dt] = {k: v.grad for k, v in P.vars.items()}
    e_gpu, e_cpu = check_grads_global({k: tr.chunk.grad_view(k) for k in grads[torch.float64]},
                                      grads[torch.float64], grads[torch.float32],
                                      GRAD_FACTOR[_lib.load().tde_get_conv_math()])
    al = gather(tr.chunk.grad)
    assert torch.equal(al[0], al[1]), "ranks hold different exchanged gradients"
    if rank == 0:
        print(f"c2_syncbn: whole-batch gradient vs fp64 oracle {e_gpu:.2e} (fp32 oracle {e_cpu:.2e})")


def case_c4_syncbn(rank, world, mode):
    from oracle import losses as OL
    from oracle import nets as ON
    from test_gpu_nets import GRAD_FACTOR, check_grads_global, oracle_params_from, rel_err
    from tf_depth_estimation_amd import _lib
    assert mode == "eager", "SyncBN over gloo all-reduces on the host: eager only"
    from test_gpu_trainers import intrinsics, small_pose, texture
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    G = 2 * B
    il, ir = texture(G, H, W, 31), texture(G, H, W, 32)
    lab = torch.tensor(np.random.default_rng(33).uniform(0.1, 2.0, (G, H, W, 1)), dtype=torch.float32)
    K, gt = intrinsics(G, H, W), small_pose(G, 34)
    sl = slice(rank * B, (rank + 1) * B)
    tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
    assert tr.twin and tr.runs["s"].groups == 2
    tr.set_batch(il[sl].cuda(), ir[sl].cuda(), lab[sl].cuda(), K[sl].cuda(), gt[sl].cuda())
    tr.enable_sync_bn(world)
    tr.enable_ddp(world, bucket_mb=4.0)
    P64 = [oracle_params_from(c, "", torch.float64) for c in tr.chunks]
    P32 = [oracle_params_from(c, "", torch.float32) for c in tr.chunks]
    tr.grad_sync.begin_step()
    tr.phase_compute()
    tr.grad_sync.finish()
    torch.cuda.synchronize()
    parts = tr.loss_parts()
    out = {k: [t.detach().cpu() for t in v] for k, v in tr._out.items()}
    pose = {d: tr.pose[d].detach().cpu() for d in ("lr", "rl")}
    vals = torch.tensor([parts[k] for k in ("smooth", "depth", "exp", "cam", "photo", "consist")], dtype=torch.float64)
    al = gather(vals)
    mean_parts = (al[0] + al[1]) / world
    grads = {}
    for dt, Ps in ((torch.float64, P64), (torch.float32, P32)):
        Pss, Ppp = Ps
        x = {"il": il.to(dt), "ir": ir.to(dt)}                 # the WHOLE batch on one device
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True,
                                   scope="model_pairdepth/depth_cam_net", levels=4)
        total, rp = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"], lab.to(dt),
                                              K.to(dt), gt.to(dt))
        if dt == torch.float64:
            for i in range(4):
                for key, ref in (("sl", dsl), ("sr", dsr), ("pl", dpl), ("pr", dpr)):
                    e = rel_err(out[key][i], ref[i][sl])
                    assert e <= 1e-4, f"rank {rank} {key} disp{i + 1}: SyncBN vs whole-batch BN {e:.2e}"
                assert rel_err(out["pl"][5 + i], ml[i][sl]) <= 1e-4 and rel_err(out["pr"][5 + i], mr[i][sl]) <= 1e-4
            assert rel_err(pose["lr"], pr.reshape(G, 6)[sl]) <= 1e-4 and rel_err(pose["rl"], pl.reshape(G, 6)[sl]) <= 1e-4

            def v(t):
                return t.item() if torch.is_tensor(t) else float(t)
            want = [v(rp["smooth"]), v(rp["depth"]), v(rp["exp"]), v(rp["cam"]), v(rp["pixel"]), v(rp["consist"])]
            for name, got, w, tol in zip(("smooth", "depth", "exp", "cam", "photo", "consist"), mean_parts.tolist(),
                                         want, (1e-5,) * 5 + (1e-4,)):
                assert abs(got - w) <= tol * abs(w) + 1e-9, (name, got, w)
        total.backward()
        grads[dt] = {n: t.grad for P in Ps for n, t in P.vars.items()}
    gpu = {}
    for c in tr.chunks:
        gpu.update({n: c.grad_view(n) for n in c.names()})
    e_gpu, e_cpu = check_grads_global(gpu, grads[torch.float64], grads[torch.float32],
                                      GRAD_FACTOR[_lib.load().tde_get_conv_math()])
    if rank == 0:
        print(f"c4_syncbn: whole-batch gradient vs fp64 oracle {e_gpu:.2e} (fp32 oracle {e_cpu:.2e})")


def main():
    case, mode = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)            # both ranks share the box's one GPU
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == 2
    torch.set_num_threads(4)
    try:
        {"c4_local": case_c4_local, "c2_syncbn": case_c2_syncbn, "c4_syncbn": case_c4_syncbn}[case](rank, world, mode)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if rank == 0:
        print(f"ddp_gpu_worker {case} {mode} ok (world {world})")


if __name__ == "__main__":
    main()
