"""Launch status of the ABI entries with a stale error in the calling thread's last-error slot.

Round 4's capture abort (gpurun_out/bench_r04s_syncbn.err): another library's hipEventQuery on an unfinished event
left hipErrorNotReady in the thread's last-error slot, and the next ABI call read it as its own launch failure.  Every
launching entry now clears the slot first (tde_clear_error, csrc/tde_common.h), so a planted stale code -- the
event query's, or an unrelated one -- must not turn a good call into TDE_ERR_HIP, and the call's result must be
right."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    from tf_depth_estimation_amd import _lib
    return _lib.hip()


def _plant_not_ready():
    """hipEventQuery on an event recorded behind a long kernel: returns (and records) hipErrorNotReady."""
    hip = _hip()
    ev = ctypes.c_void_p()
    assert hip.hipEventCreate(ctypes.byref(ev)) == 0
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.cuda._sleep(50_000_000)
    assert hip.hipEventRecord(ev, st) == 0
    rc = hip.hipEventQuery(ev)
    return ev, rc


def _plant_invalid_device():
    """hipSetDevice on a device that does not exist: hipErrorInvalidDevice in the slot, current device unchanged."""
    return _hip().hipSetDevice(ctypes.c_int(9999))


@pytest.mark.parametrize("plant", ["not_ready", "invalid_device"])
def test_stale_error_is_not_read_as_a_launch_failure(plant):
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    x = torch.zeros(4096, device="cuda")
    y = torch.ones(4096, device="cuda")
    ev = None
    if plant == "not_ready":
        ev, rc = _plant_not_ready()
        assert rc != 0, "the event finished before the query: no stale code planted"
    else:
        assert _plant_invalid_device() != 0
    st = _lib.stream_ptr()
    assert lib.tde_fill(x.numel(), _lib.ptr(x), 3.0, st) == 0          # TDE_OK despite the stale code
    assert lib.tde_scale(y.numel(), _lib.ptr(y), 0.5, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(x, torch.full_like(x, 3.0))
    assert torch.equal(y, torch.full_like(y, 0.5))
    if ev is not None:
        _hip().hipEventDestroy(ev)
    _hip().hipGetLastError()
