"""GPU parity of the inference pre/post-processing kernels (csrc/postproc.hip) with the NumPy restatement of
OpenCV's algorithms (oracle/cv_ops.py) -- batch_prediction.py:62 (INTER_AREA input resize), :72 (INTER_CUBIC
resize of the disparity) and :73 (bilateralFilter 9 / 75 / 75).  Against cv2 itself: parity unpinned (not vendored,
not importable).  Bars: uint8 results and the cubic resize bit-exact (same float operations in the same order, no
FMA contraction); the bilateral filter within 2e-6 of the map's range (its 4096-bin colour table comes from
exp() evaluated by the device's libm vs the host's)."""
import numpy as np
import pytest
import torch

from oracle import cv_ops as C

pytestmark = pytest.mark.gpu


def _u8(rng, *shape):
    return rng.integers(0, 256, shape, dtype=np.uint8)


@pytest.mark.parametrize("H,W,OH,OW,Cc", [
    (60, 90, 24, 36, 3),      # non-integer down-scale (2.5): area tables
    (48, 64, 24, 32, 3),      # integer factor 2: the box mean
    (45, 45, 15, 15, 1),      # integer factor 3, one channel
    (20, 30, 24, 36, 3),      # up-scale: area-emulating fixed-point linear path
    (40, 20, 24, 36, 3),      # y down, x up: the emulation path on both axes
    (70, 50, 24, 24, 4),      # ragged non-integer scales, 4 channels
    (24, 36, 24, 36, 3),      # same size: a copy
])
def test_resize_area_u8_matches_oracle(H, W, OH, OW, Cc):
    from tf_depth_estimation_amd import batch_prediction as BP
    rng = np.random.default_rng(H * 131 + W)
    img = _u8(rng, 2, H, W, Cc)
    dev = torch.from_numpy(img).cuda()
    f32 = torch.full((2, OH, OW, Cc + 1), -7.0, device="cuda")       # a padded channel view (cstride C + 1)
    out = BP.resize_area(dev, OH, OW)
    BP.resize_area(dev, OH, OW, out_f32=f32)
    torch.cuda.synchronize()
    for b in range(2):
        ref = C.resize_area_u8(img[b], OH, OW)
        assert np.array_equal(out[b].cpu().numpy(), ref), (b, int((out[b].cpu().numpy() != ref).sum()))
        assert np.array_equal(f32[b, ..., :Cc].cpu().numpy(), ref.astype(np.float32))
    assert torch.all(f32[..., Cc] == -7.0), "the pad channel was written"


@pytest.mark.parametrize("H,W,OH,OW", [(32, 48, 60, 100), (64, 96, 30, 50), (56, 56, 240, 720), (17, 23, 17, 23)])
def test_resize_cubic_matches_oracle(H, W, OH, OW):
    from tf_depth_estimation_amd import batch_prediction as BP
    rng = np.random.default_rng(H + W)
    maps = rng.uniform(0.01, 5.0, (2, H, W, 2)).astype(np.float32)    # channel 0 of a 2-channel view
    dev = torch.from_numpy(maps).cuda()
    out = BP.resize_cubic(dev[..., :1], OH, OW)
    torch.cuda.synchronize()
    for b in range(2):
        ref = C.resize_cubic(maps[b, :, :, 0], OH, OW)
        got = out[b].cpu().numpy()
        assert np.array_equal(got, ref), float(np.abs(got - ref).max())


@pytest.mark.parametrize("d,sc,ss", [(9, 75.0, 75.0), (9, 0.3, 75.0), (5, 0.05, 2.0), (0, 1.0, 2.0)])
def test_bilateral_matches_oracle(d, sc, ss):
    from tf_depth_estimation_amd import batch_prediction as BP
    rng = np.random.default_rng(d + int(sc * 10))
    yy, xx = np.meshgrid(np.arange(40), np.arange(60), indexing="ij")
    maps = np.stack([(np.sin(0.2 * xx) + 0.5 * np.cos(0.15 * yy) + 0.05 * rng.standard_normal((40, 60))),
                     (xx > 30) * 1.0 + 0.02 * rng.standard_normal((40, 60))]).astype(np.float32)
    dev = torch.from_numpy(maps).cuda()
    out = BP.bilateral_filter(dev, d, sc, ss)
    torch.cuda.synchronize()
    for b in range(2):
        ref = C.bilateral(maps[b], d, sc, ss)
        got = out[b].cpu().numpy()
        span = float(maps[b].max() - maps[b].min())
        assert np.abs(got - ref).max() <= 2e-6 * span, float(np.abs(got - ref).max())


def test_bilateral_constant_map_is_copied():
    from tf_depth_estimation_amd import batch_prediction as BP
    z = torch.full((1, 16, 20), 0.75, device="cuda")
    assert torch.equal(BP.bilateral_filter(z), z)


def test_predict_depth_map_pipeline():
    """batch_prediction.py:58-75 for one decoded image: INTER_AREA into the network input, the folded-BN disp_net
    graph, INTER_CUBIC of disp1 to (image_height, image_width) and the 9 / 75 / 75 bilateral filter.  The network
    input equals the oracle's area resize of the image (float of the uint8 values), and z equals the oracle's
    cubic + bilateral of the GPU's own disp1 (the network itself: tests/test_gpu_inference.py)."""
    from tf_depth_estimation_amd import _api, batch_prediction as BP, variables
    variables.get_store().reset(seed=3)
    _api.clear_programs()
    pr = BP.Predictor("disp_net", 64, 64)
    rng = np.random.default_rng(9)
    img = _u8(rng, 90, 130, 3)
    z = pr.predict_depth_map(torch.from_numpy(img), out_hw=(48, 144))
    torch.cuda.synchronize()
    assert np.array_equal(pr.x[0].cpu().numpy(), C.resize_area_u8(img, 64, 64).astype(np.float32))
    disp1 = pr.outs[0][0, :, :, 0].cpu().numpy()
    ref = C.bilateral(C.resize_cubic(disp1, 48, 144), 9, 75.0, 75.0)
    got = z[0].cpu().numpy()
    assert got.shape == (48, 144)
    assert np.abs(got - ref).max() <= 2e-6 * max(float(np.abs(ref).max()), 1e-6)
    _api.clear_programs()


def test_predict_pose_pipeline_and_11_channel_depth_net():
    """batch_prediction_cam_est.py:79-98: two uint8 images INTER_AREA-resized into the halves of the 6-channel input,
    then depth_net's pose; and batch_prediction_optflow.py:43's 11-channel depth_net input (Predictor(cin=11))."""
    from tf_depth_estimation_amd import _api, batch_prediction as BP, variables
    variables.get_store().reset(seed=4)
    _api.clear_programs()
    pr = BP.Predictor("depth_net", 64, 96)
    rng = np.random.default_rng(12)
    a, b = _u8(rng, 120, 200, 3), _u8(rng, 100, 150, 3)
    pose = pr.predict_pose(torch.from_numpy(a), torch.from_numpy(b)).clone()
    torch.cuda.synchronize()
    x = pr.x[0].cpu().numpy()
    assert np.array_equal(x[..., :3], C.resize_area_u8(a, 64, 96).astype(np.float32))
    assert np.array_equal(x[..., 3:], C.resize_area_u8(b, 64, 96).astype(np.float32))
    again = pr(pr.x.clone())[2].reshape(1, 6)
    assert torch.equal(pose, again) and pose.shape == (1, 6)
    _api.clear_programs()
    variables.get_store().reset(seed=5)
    p11 = BP.Predictor("depth_net", 64, 96, cin=11, scope="model11")
    assert p11.x.shape == (1, 64, 96, 11)
    outs = p11(torch.rand(1, 64, 96, 11, device="cuda"))
    assert all(torch.isfinite(o).all() for o in outs)
    assert p11.prog.chunk.view("model11/depth_cam_net/cnv1/weights").shape[2] == 11
    _api.clear_programs()
