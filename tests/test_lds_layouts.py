"""LDS layout checks of the halo conv (halo_conv.hip, CPU-only): the XOR-swizzled compact halo rows the fp16x3 planner
picks for 24 / 32 / 56 / 64-channel chunks are never worse than the padded rows they replace for the ds_read_b128
fragment reads of every tap shift (gfx950 lane groups, MI355X_MICROARCH.md LDS table), conflict-free where the padded
rows were, and take less LDS per halo row.  The model is scripts/halo_swizzle_check.py's."""
import functools
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@functools.lru_cache(maxsize=1)
def _model():
    spec = importlib.util.spec_from_file_location("halo_swz", os.path.join(ROOT, "scripts", "halo_swizzle_check.py"))
    mod = importlib.util.module_from_spec(spec)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        spec.loader.exec_module(mod)
    return mod


def planner_layout(cc):
    """(SA, swizzle) as halo_plan picks them for a channel chunk of cc (fp16x3)."""
    M = _model()
    sa = M.lds_stride(cc)
    if 16 < cc <= 32 and sa > 32:
        return 32, lambda r: (r >> 1) & 3
    if 32 < cc <= 64 and sa > 64:
        return 64, lambda r: r & 7
    return sa, None


@pytest.mark.parametrize("cc,k", [(32, 7), (32, 3), (32, 5), (24, 3), (24, 7), (64, 5), (64, 3), (56, 3)])
def test_swizzled_halo_rows_no_worse(cc, k):
    M = _model()
    HWd = 16 + k - 1
    sa0 = M.lds_stride(cc)
    padded = lambda r, c: r * sa0 * 2 + 16 * c
    sa, f = planner_layout(cc)
    assert f is not None and sa < sa0
    swz = lambda r, c: r * sa * 2 + 16 * (c ^ f(r))
    w_pad = M.read_worst(cc, k, k, HWd, sa0, padded)
    w_swz = M.read_worst(cc, k, k, HWd, sa, swz)
    assert w_swz <= w_pad
    if cc in (32, 64):
        assert w_swz == 1          # chunk-aligned taps: conflict-free, as the padded rows were
