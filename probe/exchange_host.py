"""Diagnostic (round 6): host-side cost of one eager gradient all-reduce at world 1 -- through ProcessGroupNCCL
(`dist.all_reduce`) and straight through RCCL (`ncclAllReduce` via ctypes on the same library torch loaded) -- and
the device time of each, for a 126 MB fp32 buffer (one config-4 network's gradient).  Prints one JSON line."""
import ctypes
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    n = 126 * 2 ** 20 // 4
    buf = torch.ones(n, device="cuda")
    side = torch.cuda.Stream()
    out = {}
    for name in ("pg", "rccl"):
        if name == "rccl":
            lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
            uid = UniqueId()
            assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
            comm = ctypes.c_void_p()
            assert lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0

            def call():
                r = lib.ncclAllReduce(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(buf.data_ptr()),
                                      ctypes.c_size_t(n), 7, 0, comm, ctypes.c_void_p(side.cuda_stream))
                assert r == 0, r
        else:
            def call():
                with torch.cuda.stream(side):
                    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        host = []
        for _ in range(20):
            t0 = time.perf_counter()
            call()
            host.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        for _ in range(20):
            call()
        e1.record(side)
        torch.cuda.synchronize()
        host.sort()
        out[name] = {"host_us_median": round(host[10] * 1e6, 1), "host_us_max": round(host[-1] * 1e6, 1),
                     "device_us_per_call": round(e0.elapsed_time(e1) * 1e3 / 20, 1)}
        print(name, out[name], flush=True)
    print(json.dumps({"probe": "eager all-reduce of 126 MB at world 1", **out}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
