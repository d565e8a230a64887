"""CPU-side checks of the drop-in boundary: libtde.so loads, exports every symbol include/tde.h
declares, and the ctypes signature table covers exactly that set.  No device calls."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "tde.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tde_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_symbols():
    syms = header_symbols()
    assert "tde_conv2d_fwd" in syms and "tde_adam_update" in syms
    assert len(syms) >= 30


def test_library_exports_every_header_symbol():
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.tde_abi_version() == _lib.ABI_VERSION


def test_ctypes_table_matches_header():
    from tf_depth_estimation_amd import _lib
    assert sorted(_lib.exported_symbols()) == header_symbols()


def test_status_strings_and_arg_checks():
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    assert lib.tde_status_string(0) == b"ok"
    assert lib.tde_status_string(-2) == b"workspace too small"
    # host-side argument validation returns before any device work
    d = _lib.ConvDesc()
    assert lib.tde_conv2d_workspace_size(ctypes.byref(d), 0) == 0
    assert lib.tde_conv2d_fwd(ctypes.byref(d), None, None, None, 0, None, 0, None) == -1
    assert lib.tde_bn_fwd_train(0, 3, 1, None, None, 1e-3, 0.99, 1, None, None, None, None, None, 4, 0, 1, None, 0,
                                None) == -1


def test_workspace_query_splits_deep_layers():
    """cnv7b-like layer at batch 8: few output tiles -> split-K workspace is requested."""
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    d = _lib.ConvDesc(N=8, H=2, W=2, C=512, OH=2, OW=2, K=512, KH=3, KW=3, stride=1, pad_top=1, pad_left=1,
                      w_cin=512, x_cstride=512, x_coff=0, y_cstride=512, y_coff=0)
    assert lib.tde_conv2d_workspace_size(ctypes.byref(d), 0) > 0


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "tf_depth_estimation_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f


def test_inference_and_sig_loss_entry_points_validate_arguments():
    """The folded-BN inference convs, the BN fold and the DeMoN sig loss reject bad arguments on the host,
    before any device work (status -1 = TDE_ERR_ARG)."""
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    d = _lib.ConvDesc()
    assert lib.tde_conv2d_fwd_bias_act(ctypes.byref(d), None, None, None, 1, None, None, 0, None) == -1
    assert lib.tde_deconv2d_fwd_bias_act(ctypes.byref(d), None, None, None, 1, None, None, 0, None) == -1
    assert lib.tde_bn_fold(0, 4, 4, 0, None, None, None, None, 1e-3, None, None, None) == -1
    assert lib.tde_bn_fold(9, 4, 4, 2, None, None, None, None, 1e-3, None, None, None) == -1
    deltas = (ctypes.c_int * 1)(2)
    weights = (ctypes.c_float * 1)(1.0)
    assert lib.tde_loss_sig_l2(1, 8, 8, None, 1, 0, None, 1, ctypes.cast(deltas, ctypes.c_void_p),
                               ctypes.cast(weights, ctypes.c_void_p), 1e-3, 1e-6, 1.0, None, None, 1, 0, None) == -1
    # relu must be 0 or 1 even with an otherwise valid descriptor
    d = _lib.ConvDesc(N=1, H=8, W=8, C=4, OH=8, OW=8, K=4, KH=3, KW=3, stride=1, pad_top=1, pad_left=1, w_cin=4,
                      x_cstride=4, x_coff=0, y_cstride=4, y_coff=0)
    assert lib.tde_conv2d_fwd_bias_act(ctypes.byref(d), None, None, None, 2, None, None, 0, None) == -1


def test_depth_pyramid_entry_point_validates_arguments():
    """tde_loss_depth_pyramid rejects, on the host: a channel offset outside its view (the kernel's
    loc * cs + co offsets assume 0 <= co < cs), a smoothness term on a scale below 3 x 3 pixels (the
    reference's reduce_mean over an empty dx2 / dy2 is NaN; tde_loss_smooth2's contract) and a depth-L1 term
    at a size not divisible by 2^s.  A valid descriptor with null device pointers for the loss accumulators
    is still rejected only for its real defects (status -1 = TDE_ERR_ARG, no device work)."""
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    buf = ctypes.create_string_buffer(64)   # any non-null address: validation returns before device work

    def desc(**kw):
        a = _lib.DepthLoss()
        a.N, a.H, a.W, a.nscales = 2, 24, 32, 4
        for s in range(4):
            a.pred[s] = ctypes.addressof(buf)
            a.grad[s] = ctypes.addressof(buf)
            a.pred_cs[s], a.pred_co[s], a.g_cs[s], a.g_co[s] = 3, 1, 2, 1
            a.smooth_w[s], a.l1_w[s] = 1.0, 1.0
        a.label = ctypes.addressof(buf)
        for k, v in kw.items():
            k, s = k.rsplit("_", 1) if k[-1].isdigit() else (k, None)
            if s is None:
                setattr(a, k, v)
            else:
                getattr(a, k)[int(s)] = v
        return a

    for bad in (dict(pred_co_2=3), dict(pred_co_0=-1), dict(g_co_1=2), dict(g_co_3=-4)):
        assert lib.tde_loss_depth_pyramid(ctypes.byref(desc(**bad)), None) == -1, bad
    # 12 x 16 at scale 3 is 1 x 2 pixels: smoothness rejected, depth-L1 alone accepted by validation
    a = desc(H=12, W=16, l1_w_3=0.0)
    assert lib.tde_loss_depth_pyramid(ctypes.byref(a), None) == -1
    # H = 26 is not divisible by 4: the scale-2 depth-L1 box is ragged
    assert lib.tde_loss_depth_pyramid(ctypes.byref(desc(H=26)), None) == -1
