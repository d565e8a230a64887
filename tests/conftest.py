import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long CPU test")
    config.addinivalue_line("markers", "rccl: initialises an RCCL process group (run after every other test)")


def pytest_collection_modifyitems(session, config, items):
    """Tests that create process-wide RCCL state (an nccl process group: communicators, ProcessGroupNCCL's watchdog
    thread, RCCL's proxy threads) run last, in their collected order, so no other test shares a process with that
    state (GPUTEST_r05 aborted inside one of them, which also hid every test collected after it)."""
    rest = [it for it in items if it.get_closest_marker("rccl") is None]
    last = [it for it in items if it.get_closest_marker("rccl") is not None]
    items[:] = rest + last


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def lib():
    """The product's C-ABI library (fails loudly if it is not built)."""
    from tf_depth_estimation_amd import _lib
    return _lib.load()
