"""The overlapped gradient exchange on the GPU, in one process: a world-size-1 RCCL group runs the
real path -- backward hooks, bucket all-reduce on the comm stream, segmented hipGraph capture and
replay -- and must leave parameters bit-identical to the single-graph trainer (all-reduce over one
rank is the identity and the scale is 1.0).  The multi-rank mean itself is covered on CPU with gloo
(tests/test_ddp.py).

These tests carry the `rccl` marker: tests/conftest.py runs them after every other GPU test, so the process-wide RCCL
state they create (communicators, ProcessGroupNCCL's watchdog thread, RCCL's proxy threads) exists only at the end of
the suite."""
import os
import socket

import numpy as np
import pytest
import torch

# an empty captured segment is dropped, not replayed (train._end_segment): the warning must not surface
pytestmark = [pytest.mark.gpu, pytest.mark.rccl, pytest.mark.filterwarnings("error:The CUDA Graph is empty")]


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    if not dist.is_initialized():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _trainer(ddp, graph, steps, wgrad=None, mode="graph"):
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    N, H, W = 2, 128, 256
    tr = train.DepthOnlyTrainer(N, H, W)
    g = np.random.default_rng(3)
    tr.set_batch(torch.tensor(g.uniform(-0.5, 0.5, (N, H, W, 3)), dtype=torch.float32).cuda(),
                 torch.tensor(g.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32).cuda())
    if wgrad is not None:
        tr.enable_wgrad_overlap(serial=(wgrad == "serial"))
    if ddp:
        gs = tr.enable_ddp(1, bucket_mb=0.5, mode=mode)
        assert len(gs.buckets) > 8
    if graph:
        tr.capture(warmup=1)
        if ddp and mode == "segments":
            assert len(tr.segments) > 4, "expected the backward to be cut at bucket launches"
        if ddp and mode == "graph":
            assert tr.segments is None and len(tr.graphs) == 1, f"{mode} mode: one graph, all-reduces captured"
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return tr.chunk.flat.clone(), tr.chunk.grad.clone()


MODES = pytest.mark.parametrize("mode", ["graph", "segments"])


@MODES
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_overlapped_exchange_world1_matches_plain(pg, graph, mode):
    """World-1 RCCL exchange == no exchange, bit for bit, eager and captured, in both exchange modes (graph: the
    bucket all-reduces captured on a forked comm branch; segments: graphs cut at launch points)."""
    p0, g0 = _trainer(False, graph, 3)
    p1, g1 = _trainer(True, graph, 3, mode=mode)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)


@MODES
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_overlapped_exchange_with_wgrad_side_stream(pg, graph, mode):
    """Filter gradients on a side stream (enable_wgrad_overlap) under the bucketed exchange: every launch
    point first joins the side stream (a bucket's last parameters come from it), and under capture the
    segments close with the side branch joined.  Bit-identical to the same split backward calls run
    serially on one stream without an exchange."""
    p0, g0 = _trainer(False, graph, 3, wgrad="serial")
    p1, g1 = _trainer(True, graph, 3, wgrad="overlap", mode=mode)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)


def test_sync_bn_world1_step_parity(pg):
    """SyncBN through the trainer (enable_sync_bn) over a world-1 RCCL group: the all-reduces are the
    identity, so the eager config-2 step must meet the same bars as the plain step against the float64
    oracle (loss 1e-5; whole gradient within the fp32 noise model of tests/test_gpu_nets.py -- the BN
    summation order differs from the fused conv+BN path, and these gradients amplify rounding).  (Capture of the
    SyncBN step: test_sync_bn_captured_config4.)"""
    from oracle import losses as OL
    from oracle import nets as ON
    from test_gpu_nets import GRAD_FACTOR, check_grads_global, oracle_params_from
    from tf_depth_estimation_amd import _api, _lib, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    N, H, W = 2, 64, 96
    tr = train.DepthOnlyTrainer(N, H, W)
    g = np.random.default_rng(4)
    x = torch.tensor(g.uniform(-0.5, 0.5, (N, H, W, 3)), dtype=torch.float32)
    lab = torch.tensor(g.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32)
    tr.set_batch(x.cuda(), lab.cuda())
    tr.enable_sync_bn(1)
    Ps = {dt: oracle_params_from(tr.chunk, "", dt) for dt in (torch.float64, torch.float32)}
    tr.phase_compute()
    torch.cuda.synchronize()
    grads = {}
    for dt, P in Ps.items():
        lr, _ = OL.loss_depth_only(ON.disp_net(P, x.to(dt), True, scope="model/depth_net"), lab.to(dt))
        lr.backward()
        grads[dt] = {k: v.grad for k, v in P.vars.items()}
        if dt == torch.float64:
            assert abs(tr.total_loss() - lr.item()) <= 1e-5 * abs(lr.item())
    check_grads_global({k: tr.chunk.grad_view(k) for k in grads[torch.float64]}, grads[torch.float64],
                       grads[torch.float32], GRAD_FACTOR[_lib.load().tde_get_conv_math()])
    variables.get_store().reset(seed=1)
    _api.clear_programs()


def _c4_trainer(ddp, graph, net_overlap, steps=2, mode="graph", bucket_mb=4.0):
    from test_gpu_trainers import intrinsics, small_pose, texture
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    B, H, W = 2, 64, 96
    tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
    lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
    tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                 torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(), small_pose(B, 4).cuda())
    tr.enable_wgrad_overlap()
    if ddp:
        gs = tr.enable_ddp(1, bucket_mb=bucket_mb, mode=mode)
        assert len(gs.buckets) > (4 if bucket_mb <= 4.0 else 1)
    if net_overlap:
        tr.enable_net_overlap()
    if graph:
        tr.capture(warmup=1)
        if ddp and net_overlap and mode == "segments":
            nseg = sum(len(segs) for w, segs in tr.ov_seq if segs is not None)
            assert nseg > len([w for w, s in tr.ov_seq if s is not None]), "backward pieces were not cut"
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return [(c.flat.clone(), c.grad.clone(), c.adam_m.clone()) for c in tr.chunks]


@MODES
@pytest.mark.parametrize("bucket_mb", [4.0, 256.0], ids=["b4", "b256"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_config4_exchange_with_net_overlap(pg, graph, bucket_mb, mode):
    """Config 4 (twin-batched programs, filter gradients on their side streams, depth_net on the second stream)
    under the bucketed exchange (world-1 RCCL group): each program's bucket launch points cut its own piece's
    graphs (segments) or fork its comm branch one level deep (graph; only that program's filter-gradient branch is
    joined first) -- the parameters, gradients and moments equal the same step without an exchange bit for bit
    (deterministic warp-loss mode; world 1: the all-reduce is the identity).  b256 = the benched default, one
    bucket per network; b4 = many mid-backward launch points."""
    ref = _c4_trainer(False, graph, True)
    for a, b in zip(ref, _c4_trainer(True, graph, True, mode=mode, bucket_mb=bucket_mb)):
        assert all(torch.equal(x, y) for x, y in zip(a, b))
    for a, b in zip(ref, _c4_trainer(True, graph, False, mode=mode, bucket_mb=bucket_mb)):
        assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_graph_exchange_refused_with_net_overlap_beyond_world1(pg):
    """with the net overlap the two networks' captured exchanges would run two communicators from two
    concurrently replayed graphs; at world > 1 that order is not fixed, so it is refused (segments mode, the default,
    is accepted).  Only the schedule check runs here (no collective is issued at world 2 on a world-1 group)."""
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    tr = train.DepthThenCamTrainer(1, 64, 96)
    gs = tr.enable_ddp(2, mode="graph")
    assert gs.grad_scale == 0.5 and all(o.grad_scale == 0.5 for o in tr.opt.opts)
    with pytest.raises(ValueError):
        tr.enable_net_overlap()
    tr2 = train.DepthThenCamTrainer(1, 64, 96)
    gs2 = tr2.enable_ddp(2)
    assert gs2.mode == "segments" and gs2.inline and all(o.grad_scale == 0.5 for o in tr2.opt.opts)
    tr2.enable_net_overlap()
    _api.clear_programs()


def _c4_syncbn(pg, graph, sync=True, steps=3, overlaps=None):
    from test_gpu_trainers import intrinsics, small_pose, texture
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    B, H, W = 2, 64, 96
    tr = train.DepthThenCamTrainer(B, H, W).enable_deterministic()
    lab = np.random.default_rng(3).uniform(0.1, 2.0, (B, H, W, 1))
    tr.set_batch(texture(B, H, W, 1).cuda(), texture(B, H, W, 2).cuda(),
                 torch.tensor(lab, dtype=torch.float32).cuda(), intrinsics(B, H, W).cuda(), small_pose(B, 4).cuda())
    if sync:
        tr.enable_sync_bn(1)
        assert tr.sync_bn_capturable
    if overlaps is not None:
        # the benched schedule (or its serial form): depth_net's filter gradients on a side stream, the two
        # networks on two streams -- each program all-reducing on a communicator of its own
        serial = overlaps == "serial"
        tr.enable_wgrad_overlap(serial=serial, only=["pair"])
        if not serial:
            tr.enable_net_overlap()
    n = steps
    if graph:
        tr.capture(warmup=1)
        n -= 1
    for _ in range(n):
        tr.step()
    torch.cuda.synchronize()
    outs = {k: [t.detach().clone() for t in v] for k, v in tr._out.items()}
    return [(c.flat.clone(), c.grad.clone(), c.adam_m.clone()) for c in tr.chunks], outs


def test_sync_bn_captured_config4(pg):
    """SyncBN over RCCL is graph-capturable: config 4 with twin batching (row-grouped SyncBN:
    each group's sums all-reduced together, on a communicator of its own) captured and replayed equals the same
    SyncBN steps run eagerly bit for bit (world-1 group, deterministic warp-loss mode; 3 steps each), and at world 1
    SyncBN is BatchNorm over the local rows: the network outputs of the step match the local-BN trainer's within the
    network-output bar, 1e-4 (different statistics kernels -- the sums pass vs the conv epilogue partials -- round
    differently, and ~30 layers carry it on: measured 1.3e-5)."""
    g_ref, o_ref = _c4_syncbn(pg, False)
    g_cap, o_cap = _c4_syncbn(pg, True)
    for a, b in zip(g_ref, g_cap):
        assert all(torch.equal(x, y) for x, y in zip(a, b)), "captured SyncBN step != eager SyncBN step"
    # the overlapped schedule under SyncBN (per-program and per-branch communicators) == its serial form
    g_ser, _ = _c4_syncbn(pg, False, overlaps="serial")
    g_ov, _ = _c4_syncbn(pg, True, overlaps="overlap")
    for a, b in zip(g_ser, g_ov):
        assert all(torch.equal(x, y) for x, y in zip(a, b)), "overlapped SyncBN step != its serial form"
    _, o_loc = _c4_syncbn(pg, False, sync=False, steps=1)
    _, o_sb1 = _c4_syncbn(pg, False, sync=True, steps=1)
    for k in o_loc:
        for a, b in zip(o_loc[k], o_sb1[k]):
            err = ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
            assert err <= 1e-4, (k, err)


def test_direct_rccl_communicator(pg):
    """rccl.Communicator (the exchange's direct RCCL path): a world-1 communicator built through the process group's
    unique-id broadcast; in-place SUM on a given stream, eagerly and captured in a hipGraph, is the identity at one
    rank; bad operands are refused on the host."""
    from tf_depth_estimation_amd import rccl
    c = rccl.Communicator()
    assert c.world == 1 and c.rank == 0 and c.comm.value
    t = torch.randn(1 << 20, device="cuda")
    ref = t.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    c.all_reduce_sum(t, s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        c.all_reduce_sum(t)      # (at one rank RCCL records no node for an in-place SUM)
        t.mul_(1.0)              # keep the graph non-empty
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    d = torch.ones(1000, dtype=torch.float64, device="cuda")      # SyncBN's fp64 sums
    c.all_reduce_sum(d)
    torch.cuda.synchronize()
    assert torch.equal(d, torch.ones_like(d))
    for bad in (t.to(torch.int32), t.view(2, -1).t(), t.cpu()):
        with pytest.raises(ValueError):
            c.all_reduce_sum(bad)
    assert rccl.pooled_comm("test", 0) is rccl.pooled_comm("test", 0)
