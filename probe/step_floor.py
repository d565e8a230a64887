"""Cost of one extra tiny kernel inside the real config-2 step: capture the step with a tde_scale(n=16)
launched after every ABI call and compare step times (diagnostic for the per-launch floor)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tf_depth_estimation_amd import _lib  # noqa: E402

lib = _lib.load()
dummy = torch.zeros(64, device="cuda")
count = [0]
orig_check = _lib.check
EXTRA = int(os.environ.get("EXTRA", "0"))


def check_with_extra(status, what=""):
    orig_check(status, what)
    for _ in range(EXTRA):
        lib.tde_scale(16, _lib.ptr(dummy), 1.0, _lib.stream_ptr())
        count[0] += 1


_lib.check = check_with_extra
tr = bench.make_trainer("config2", 8)
tr.set_batch(*[t.cuda() for t in bench.make_batch("config2", 8, 0)])
count[0] = 0
tr.capture()
n_extra = count[0]
for _ in range(10):
    tr.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    tr.step()
torch.cuda.synchronize()
print(f"EXTRA={EXTRA} extra kernels captured ~{n_extra // 3} per step; {1e3 * (time.perf_counter() - t0) / 50:.3f} ms/step")
