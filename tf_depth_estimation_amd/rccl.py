"""Direct RCCL communicators for the gradient exchange: `ncclAllReduce` issued straight on the
caller's HIP stream through ctypes, on the same librccl torch loaded -- no ProcessGroupNCCL in the data path.

Why not `torch.distributed.all_reduce` for the exchange (round 6):
  * ProcessGroupNCCL wraps every call in Work objects, events and a watchdog thread that polls them; the one SIGABRT
    on record in this code base is that watchdog terminating on an event recorded inside a stream capture
    (DESIGN.md §5).  A direct call creates no event and nothing polls it, eager or captured;
  * its eager call costs ~14 us of host time and ~16 us of device time per collective at world 1 against 0.8 us /
    0.5 us for the direct call (probe/exchange_host.py, profiles/r06/xhost.txt);
  * it issues on the current stream or its own internal stream; a direct call goes exactly where the caller says --
    here the stream of the network whose gradients it reduces, so no extra stream (a fifth stream shares one of
    GPU_MAX_HW_QUEUES = 4 FIFO hardware queues with a compute chain and stalled it: -28 % at world 1).

A communicator is created collectively: rank 0 of the process group draws an `ncclUniqueId`, every rank receives it
with `torch.distributed.broadcast_object_list` over that group (setup only, eager), then `ncclCommInitRank`.  All
ranks create communicators in the same order (pooled by purpose and index, `pooled_comm`).
"""
import ctypes
import os

import torch

NCCL_FLOAT32 = 7     # ncclDataType_t ncclFloat32
NCCL_FLOAT64 = 8     # ncclDataType_t ncclFloat64
NCCL_SUM = 0         # ncclRedOp_t ncclSum
_DTYPES = {torch.float32: NCCL_FLOAT32, torch.float64: NCCL_FLOAT64}

_LIB = None


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]     # NCCL_UNIQUE_ID_BYTES


def lib():
    """librccl.so as torch loaded it (one RCCL instance per process)."""
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        L = ctypes.CDLL(path)
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        L.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        L.ncclGetErrorString.argtypes = [ctypes.c_int]
        _LIB = L
    return _LIB


class RcclError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise RcclError(f"{what}: RCCL error {rc} ({lib().ncclGetErrorString(rc).decode()})")


class Communicator:
    """An RCCL communicator over the ranks of `group` (the default process group when None)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        # the id as its raw 128 bytes (a c_char array field reads back only up to its first NUL byte)
        box = [ctypes.string_at(ctypes.addressof(uid), 128) if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(box, src=src, group=group)
        if len(box[0]) != 128:
            raise RcclError("ncclUniqueId broadcast: expected 128 bytes")
        raw = ctypes.create_string_buffer(box[0], 128)
        ctypes.memmove(ctypes.addressof(uid), raw, 128)
        self.comm = ctypes.c_void_p()
        _check(lib().ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank), "ncclCommInitRank")

    def all_reduce_sum(self, t, stream=None):
        """In-place SUM over the ranks of a contiguous float32 / float64 CUDA tensor (gradients / SyncBN's fp64 sums),
        issued on `stream` (default: the current stream).  Stream-ordered, no host synchronisation, capturable."""
        if t.dtype not in _DTYPES or not t.is_cuda or not t.is_contiguous():
            raise ValueError("all_reduce_sum expects a contiguous float32 or float64 CUDA tensor")
        st = (stream or torch.cuda.current_stream()).cuda_stream
        _check(lib().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPES[t.dtype], NCCL_SUM, self.comm,
                                   ctypes.c_void_p(st)), "ncclAllReduce")


_POOL = {}


def pooled_comm(purpose, idx, group=None):
    """The idx-th communicator of `purpose` over `group`, created on first use and reused by later trainers of this
    process (all ranks ask in the same order).  Entries hold the process group they were made under, so a
    re-initialised default group gets fresh ones."""
    import torch.distributed as dist
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    key = (id(pg), purpose, idx)
    hit = _POOL.get(key)
    if hit is None:
        hit = _POOL[key] = (pg, Communicator(group))
    return hit[1]
