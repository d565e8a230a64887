"""World size 2 ON the GPU: two data-parallel ranks sharing the box's one MI355X, launched by
torch.distributed.run before any GPU call, with the gloo backend (one card cannot host two RCCL ranks; the exchange
code path -- bucket hooks, comm stream, event waits, segmented capture and replay -- is the same one bench.py --gpus N
runs over RCCL).  tests/ddp_gpu_worker.py holds the cases and their assertions:

  c4_local (eager, graph): config 4 with twin batching, net overlap, filter-gradient streams and the bucketed
      exchange; exchanged gradient == mean of the ranks' local gradients bit for bit, within the oracle bars of the
      mean of the fp64 per-shard gradients, replicas bit-identical after Adam and over later (replayed) steps;
  c2_syncbn (eager): SyncBN across the two ranks == whole-batch BatchNorm (outputs 1e-4, loss 1e-5, gradient within
      the oracle bars of the whole-batch fp64 gradient);
  c4_syncbn (eager): the same for config 4's twin-batched, row-grouped SyncBN (each call's BatchNorm batch spans both
      ranks: the reference's one-device batch of 2B)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("case,mode", [("c4_local", "eager"), ("c4_local", "graph"), ("c2_syncbn", "eager"),
                                       ("c4_syncbn", "eager")])
def test_two_ranks_on_one_gpu(case, mode):
    env = dict(os.environ, OMP_NUM_THREADS="4", PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "ddp_gpu_worker.py"), case, mode]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    print(r.stdout[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert f"ddp_gpu_worker {case} {mode} ok (world 2)" in r.stdout
