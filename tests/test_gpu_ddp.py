"""The overlapped gradient exchange on the GPU, in one process: a world-size-1 RCCL group runs the
real path -- backward hooks, bucket all-reduce on the comm stream, segmented hipGraph capture and
replay -- and must leave parameters bit-identical to the single-graph trainer (all-reduce over one
rank is the identity and the scale is 1.0).  The multi-rank mean itself is covered on CPU with gloo
(tests/test_ddp.py)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


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


def _trainer(ddp, graph, steps):
    from tf_depth_estimation_amd import _api, train, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    N, H, W = 2, 128, 256
    tr = train.DepthOnlyTrainer(N, H, W)
    g = np.random.default_rng(3)
    tr.set_batch(torch.tensor(g.uniform(-0.5, 0.5, (N, H, W, 3)), dtype=torch.float32).cuda(),
                 torch.tensor(g.uniform(0.25, 4.0, (N, H, W, 1)), dtype=torch.float32).cuda())
    if ddp:
        gs = tr.enable_ddp(1, bucket_mb=0.5)
        assert len(gs.buckets) > 8
    if graph:
        tr.capture(warmup=1)
        if ddp:
            assert len(tr.segments) > 4, "expected the backward to be cut at bucket launches"
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return tr.chunk.flat.clone(), tr.chunk.grad.clone()


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_overlapped_exchange_world1_matches_plain(pg, graph):
    p0, g0 = _trainer(False, graph, 3)
    p1, g1 = _trainer(True, graph, 3)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)
