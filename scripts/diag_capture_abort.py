"""Diagnostic (round 6): repeat the config-4 captured exchange + net overlap capture of
tests/test_gpu_ddp.py::test_config4_exchange_with_net_overlap[graph-*] in ONE process with full stderr, so an
intermittent abort (GPUTEST_r05: SIGABRT inside Trainer.capture) leaves its message.  Not a test."""
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
faulthandler.enable(all_threads=True)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    mode = sys.argv[2] if len(sys.argv) > 2 else "graph"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from test_gpu_ddp import _c4_trainer
    for i in range(reps):
        t0 = time.time()
        ref = _c4_trainer(False, True, True)
        got = _c4_trainer(True, True, True, mode=mode)
        ok = all(torch.equal(x, y) for a, b in zip(ref, got) for x, y in zip(a, b))
        print(f"rep {i} mode={mode} equal={ok} {time.time() - t0:.1f}s", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
