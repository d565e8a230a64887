"""Inference path (batch_prediction*.py): BN folded into the convs, one bias+ReLU
conv launch per layer, hipGraph-captured batch predictor -- against the float64 oracle in inference
mode (is_training=False: moving statistics) on identical inputs.

Tolerances: kernels 1e-5 relative-to-max (as tests/test_gpu_kernels.py); network outputs 1e-4 (the
north-star bar).  Moving statistics are randomised so the fold is exercised with non-trivial scales."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import nets as ON
from oracle import tf_ops as T
from test_gpu_kernels import close, conv_desc, dev, rnd, ws_for  # noqa: F401  (dev's autouse fixture)
from test_gpu_kernels import _release_temps  # noqa: F401
from test_gpu_nets import images, oracle_params_from, rel_err

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4


@pytest.fixture(scope="module")
def L():
    from tf_depth_estimation_amd import _lib
    return _lib


@pytest.fixture
def fresh_store():
    from tf_depth_estimation_amd import _api, variables
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    yield
    variables.get_store().reset(seed=1)
    _api.clear_programs()


@pytest.mark.parametrize("layout", [0, 1], ids=["conv", "deconv"])
def test_bn_fold(L, layout):
    lib = L.load()
    k, cin, K = 3, 12, 8
    shape = (k, k, cin, K) if layout == 0 else (k, k, K, cin)
    w = rnd(*shape, seed=1)
    mm, beta = rnd(K, seed=2), rnd(K, seed=3)
    mv = rnd(K, seed=4, lo=0.1, hi=3.0)
    wf = torch.empty(shape, device="cuda")
    bf = torch.empty(K, device="cuda")
    L.check(lib.tde_bn_fold(k * k, cin, K, layout, L.ptr(dev(w)), L.ptr(dev(mm)), L.ptr(dev(mv)), L.ptr(dev(beta)),
                            1e-3, L.ptr(wf), L.ptr(bf), L.stream_ptr()))
    s = 1.0 / torch.sqrt(mv.float().double() + 1e-3)
    ref = w.float().double() * (s if layout == 0 else s[:, None])
    close(wf, ref, tol=1e-6, what="folded weights")
    close(bf, beta.float().double() - mm.float().double() * s, tol=1e-6, what="folded bias")


BIAS_ACT_CASES = [
    # N, H, W, C, K, k, s, y_cs, y_coff   (plan exercised)
    (2, 24, 32, 4, 32, 7, 2, 36, 4),         # cnv1-like, direct epilogue, offset view
    (2, 2, 2, 512, 512, 3, 1, 1024, 512),    # skinny weight-streaming kernel
    (4, 24, 32, 256, 128, 3, 1, 128, 0),     # split-K: bias/ReLU in the reduce
    (3, 13, 17, 32, 64, 5, 2, 64, 0),        # ragged tiles
    (8, 6, 8, 256, 512, 3, 2, 512, 0),       # skinny at stride 2
    (2, 96, 128, 32, 32, 7, 1, 32, 0),       # halo path (bf16x6 modes)
    (1, 120, 140, 132, 64, 3, 1, 68, 4),     # halo, 3 channel chunks, offset output view
]


@pytest.mark.parametrize("case", BIAS_ACT_CASES)
@pytest.mark.parametrize("relu", [1, 0])
def test_conv2d_fwd_bias_act(L, case, relu):
    lib = L.load()
    N, H, W, C, K, k, s, ycs, yco = case
    OH, pt, _ = T.same_pad(H, k, s)
    OW, pl, _ = T.same_pad(W, k, s)
    d = conv_desc(L, N=N, H=H, W=W, C=C, OH=OH, OW=OW, K=K, KH=k, KW=k, stride=s, pad_top=pt, pad_left=pl,
                  w_cin=C, x_cstride=C, x_coff=0, y_cstride=ycs, y_coff=yco)
    x = rnd(N, H, W, C, seed=11)
    w = rnd(k, k, C, K, seed=12) * 0.2
    b = rnd(K, seed=13)
    base = rnd(N, OH, OW, ycs, seed=14)
    gy = dev(base)
    ws = ws_for(L, d)
    L.check(lib.tde_conv2d_fwd_bias_act(ctypes.byref(d), L.ptr(dev(x)), L.ptr(dev(w)), L.ptr(dev(b)), relu,
                                        L.ptr(gy), L.ptr(ws), ws.numel() * 4, L.stream_ptr()))
    ref = T.conv2d_same(x, w, s) + b
    if relu:
        ref = ref.clamp_min(0.0)
    close(gy[..., yco:yco + K], ref, what="conv bias+act")
    close(gy[..., :yco], base[..., :yco], what="view untouched lo")
    close(gy[..., yco + K:], base[..., yco + K:], what="view untouched hi")


DECONV_BIAS_CASES = [
    # N, h, w, Cin, Cout, k, view cstride, coff
    (2, 6, 8, 32, 16, 3, 36, 20),
    (2, 2, 2, 512, 512, 3, 512, 0),
    (1, 12, 16, 256, 128, 3, 128, 0),
    (2, 3, 4, 64, 32, 7, 32, 0),
    (8, 1, 1, 512, 512, 3, 1024, 0),       # upcnv7-like, split-K over the parity classes
]


@pytest.mark.parametrize("case", DECONV_BIAS_CASES)
def test_deconv2d_fwd_bias_act(L, case):
    lib = L.load()
    N, h, w_, cin, cout, k, xcs, xco = case
    H, W = 2 * h, 2 * w_
    _, pt, _ = T.same_pad(H, k, 2)
    _, pl, _ = T.same_pad(W, k, 2)
    d = conv_desc(L, N=N, H=H, W=W, C=cout, OH=h, OW=w_, K=cin, KH=k, KW=k, stride=2, pad_top=pt, pad_left=pl,
                  w_cin=cout, x_cstride=xcs, x_coff=xco, y_cstride=cin, y_coff=0)
    x = rnd(N, h, w_, cin, seed=15)
    wt = rnd(k, k, cout, cin, seed=16) * 0.2
    b = rnd(cout, seed=17)
    base = rnd(N, H, W, xcs, seed=18)
    gy = dev(base)
    ws = ws_for(L, d, deconv=True)
    L.check(lib.tde_deconv2d_fwd_bias_act(ctypes.byref(d), L.ptr(dev(x)), L.ptr(dev(wt)), L.ptr(dev(b)), 1,
                                          L.ptr(gy), L.ptr(ws), ws.numel() * 4, L.stream_ptr()))
    ref = (T.conv2d_transpose_same(x, wt, 2) + b).clamp_min(0.0)
    close(gy[..., xco:xco + cout], ref, what="deconv bias+act")
    close(gy[..., :xco], base[..., :xco], what="view untouched lo")
    close(gy[..., xco + cout:], base[..., xco + cout:], what="view untouched hi")


def randomize_moving_stats(chunk, seed, var=(0.05, 0.3)):
    """Random moving statistics near the scale of these nets' pre-BN activations, random betas (zero at
    init) so the folded bias is exercised."""
    g = np.random.default_rng(seed)
    with torch.no_grad():
        for bn_name in chunk.bn_offsets:
            m, v = chunk.moving(bn_name)
            m.copy_(torch.tensor(g.uniform(-0.05, 0.05, m.numel()), dtype=torch.float32))
            v.copy_(torch.tensor(g.uniform(*var, v.numel()), dtype=torch.float32))
        for name in chunk.names():
            if name.endswith("BatchNorm/beta"):
                t = chunk.view(name)
                t.copy_(torch.tensor(g.uniform(-0.1, 0.1, t.numel()), dtype=torch.float32))


def calibrate(chunk, x, seed, oracle_fn):
    """Moving statistics = the batch statistics of x (oracle training-mode pass with decay 0), so the
    inference activations keep unit scale through all layers: no saturated heads, and no random-scale
    growth that would make the comparison ill-conditioned.  x should hold >= 8 images: at one image the
    1x1 deep levels get a zero variance and inference BN then amplifies any input change by 1/sqrt(eps)."""
    randomize_moving_stats(chunk, seed)
    P = oracle_params_from(chunk, "")
    oracle_fn(P, x.double())
    with torch.no_grad():
        for bn_name, st in P.bn.items():
            m, v = chunk.moving(bn_name)
            m.copy_(st.moving_mean.float())
            v.copy_(st.moving_variance.float())


def calibrate_disp_net(chunk, x, seed):
    calibrate(chunk, x, seed, lambda P, x: ON.disp_net(P, x, True, scope="model/depth_net", decay=0.0))


@pytest.mark.parametrize("graph", [True, False], ids=["graph", "eager"])
def test_predictor_disp_net_parity(fresh_store, graph):
    from tf_depth_estimation_amd import batch_prediction as bp
    from tf_depth_estimation_amd import nets_optflow_depth as nod
    from tf_depth_estimation_amd import variables
    N, H, W = 2, 96, 128
    pred = bp.Predictor("disp_net", H, W, batch=N, graph=graph)
    chunk = pred.prog.chunk
    calibrate_disp_net(chunk, images(8, H, W, 3, 5), 5)
    pred.refresh()
    P = oracle_params_from(chunk, "")
    for seed in (6, 7):                                   # two replays with different inputs
        x = images(N, H, W, 3, seed)
        outs = [o.clone() for o in pred(x.cuda())]
        ref = ON.disp_net(P, x.double(), False, scope="model/depth_net")
        assert len(outs) == 4
        for i, (o, r) in enumerate(zip(outs, ref)):
            e = rel_err(o, r)
            assert e <= OUT_TOL, f"disp{i + 1} (input {seed}): rel err {e:.2e}"
            assert r.std().item() > 1e-3 * r.abs().max().item(), "degenerate (saturated) outputs"
    # the unfolded inference path (conv -> BN(moving) -> ReLU) agrees too
    with variables.variable_scope("model"):
        unf = nod.disp_net(x.cuda(), is_training=False)[0]
    for o, u in zip(outs, unf):
        assert rel_err(o, u) <= OUT_TOL


def test_predictor_depthflow_and_depth_net_parity(fresh_store):
    from tf_depth_estimation_amd import batch_prediction as bp
    N, H, W = 1, 96, 128
    x = images(N, H, W, 6, 8)
    pf = bp.Predictor("depthflow_net", H, W, batch=N)
    calibrate(pf.prog.chunk, images(8, H, W, 6, 9), 9,
              lambda P, x: ON.disp_net_depthflow(P, x, True, scope="model/depth_net", decay=0.0))
    pf.refresh()
    outs = [o.clone() for o in pf(x.cuda())]
    ref = ON.disp_net_depthflow(oracle_params_from(pf.prog.chunk, ""), x.double(), False, scope="model/depth_net")
    assert len(outs) == 8
    for i, (o, r) in enumerate(zip(outs, ref)):
        assert rel_err(o, r) <= OUT_TOL, f"depthflow output {i}"
    pd = bp.Predictor("depth_net", H, W, batch=N)
    calibrate(pd.prog.chunk, images(8, H, W, 6, 10), 10,
              lambda P, x: ON.depth_net(P, x, True, scope="model/depth_cam_net", levels=2, decay=0.0))
    pd.refresh()
    outs = [o.clone() for o in pd(x.cuda())]
    rd, rp, rm = ON.depth_net(oracle_params_from(pd.prog.chunk, ""), x.double(), False,
                              scope="model/depth_cam_net", levels=2)
    for o, r in zip(outs[:2], rd):
        assert rel_err(o, r) <= OUT_TOL
    assert rel_err(outs[2], rp) <= OUT_TOL
    for o, r in zip(outs[3:], rm):
        assert rel_err(o, r) <= OUT_TOL


def test_predictor_restore_checkpoint(fresh_store, tmp_path):
    """batch_prediction.py:49-55: build, restore a saved bundle, predict -- identical outputs."""
    from tf_depth_estimation_amd import _api, batch_prediction as bp, checkpoint, variables
    N, H, W = 1, 64, 96
    x = images(N, H, W, 3, 11).cuda()
    p1 = bp.Predictor("disp_net", H, W, batch=N)
    calibrate_disp_net(p1.prog.chunk, images(8, H, W, 3, 13), 12)
    p1.refresh()
    ref = [o.clone() for o in p1(x)]
    torch.cuda.synchronize()
    prefix = checkpoint.Saver().save(None, str(tmp_path / "model"), global_step=1)
    variables.get_store().reset(seed=99)
    _api.clear_programs()
    p2 = bp.Predictor("disp_net", H, W, batch=N)
    assert not torch.equal(p2(x)[0], ref[0])
    p2.restore(prefix)
    for a, b in zip(p2(x), ref):
        assert torch.equal(a, b)


def test_predictor_rejects_bad_shapes(fresh_store):
    from tf_depth_estimation_amd import batch_prediction as bp
    p = bp.Predictor("disp_net", 64, 96, batch=1, graph=False)
    with pytest.raises(ValueError):
        p(torch.zeros(2, 64, 96, 3, device="cuda"))
    with pytest.raises(ValueError):
        bp.Predictor("pose_exp_net", 64, 96)
