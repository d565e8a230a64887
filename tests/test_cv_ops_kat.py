"""Known-answer tests of oracle/cv_ops.py, the NumPy restatement of batch_prediction.py:62,72-73's OpenCV calls
(cv2 is not vendored by the reference and not importable here: these pin the restatement to the published
formulas -- box means, partition of unity, pixel replication, an independent float64 cubic resampler, the
bilateral filter's limits -- not to cv2)."""
import math

import numpy as np
import pytest

from oracle import cv_ops as C


def test_area_integer_factor_is_the_box_mean_rounded_to_even():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (8, 12, 3), dtype=np.uint8)
    out = C.resize_area_u8(img, 4, 6)
    box = img.reshape(4, 2, 6, 2, 3).astype(np.float64).mean(axis=(1, 3))
    assert np.array_equal(out, np.clip(np.rint(box), 0, 255).astype(np.uint8))
    # ties go to even (cvRound): a 2x2 cell summing to 10 averages 2.5 -> 2, to 6 -> 1.5 -> 2
    t = np.array([[[3], [3]], [[2], [2]]], np.uint8)
    assert C.resize_area_u8(t, 1, 1)[0, 0, 0] == 2
    t = np.array([[[1], [2]], [[1], [2]]], np.uint8)
    assert C.resize_area_u8(t, 1, 1)[0, 0, 0] == 2


@pytest.mark.parametrize("ss,ds", [(10, 4), (90, 36), (224, 224 - 31), (7, 3)])
def test_area_table_is_a_partition_of_unity(ss, ds):
    scale = ss / ds
    for taps in C._area_tab(ss, ds, 1.0 / (ds / ss)):
        assert abs(sum(float(a) for _, a in taps) - 1.0) < 1e-5
        assert all(0 <= s < ss for s, _ in taps)
    # every source index is covered, in increasing order per destination
    cov = sorted({s for taps in C._area_tab(ss, ds, scale) for s, _ in taps})
    assert cov == list(range(ss))


def test_area_constant_and_identity():
    img = np.full((33, 47, 3), 77, np.uint8)
    for oh, ow in ((10, 20), (33, 47), (50, 60), (20, 60)):
        assert np.all(C.resize_area_u8(img, oh, ow) == 77), (oh, ow)
    rng = np.random.default_rng(1)
    x = rng.integers(0, 256, (9, 11, 1), dtype=np.uint8)
    assert np.array_equal(C.resize_area_u8(x, 9, 11), x)


def test_area_upscale_reproduces_pixels_at_integer_factor():
    """Area-mode upscaling by 2 (the linear emulation): fx = (dx+1) - (sx+1)/2 is 0 or 0.5 -> 0 after the
    fractional step, so each source pixel is replicated into a 2x2 block."""
    rng = np.random.default_rng(2)
    x = rng.integers(0, 256, (5, 7, 3), dtype=np.uint8)
    out = C.resize_area_u8(x, 10, 14)
    assert np.array_equal(out, np.repeat(np.repeat(x, 2, 0), 2, 1))


def test_cubic_coefficients():
    for x in (0.0, 0.25, 0.5, 0.9):
        c = [float(v) for v in C._cubic_coeffs(x)]
        A = -0.75
        ref = [((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A,
               ((A + 2) * x - (A + 3)) * x * x + 1,
               ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1]
        ref.append(1 - sum(ref))
        assert np.allclose(c, ref, atol=1e-6)
    assert [float(v) for v in C._cubic_coeffs(0.0)] == [0.0, 1.0, 0.0, 0.0]


def test_cubic_constant_resampler_and_identity():
    z = np.full((12, 16), 3.25, np.float32)
    assert np.allclose(C.resize_cubic(z, 30, 50), 3.25, rtol=1e-6)
    # an independent float64 restatement of the separable resampling (Keys kernel with a = -0.75, which reproduces
    # constants but not ramps: only a = -0.5 does), edge taps replicated: pins the tap indexing and coefficients
    rng = np.random.default_rng(5)
    x = rng.standard_normal((11, 13)).astype(np.float32)

    def keys(t, a=-0.75):
        t = abs(t)
        if t <= 1:
            return (a + 2) * t ** 3 - (a + 3) * t ** 2 + 1
        if t < 2:
            return a * t ** 3 - 5 * a * t ** 2 + 8 * a * t - 4 * a
        return 0.0

    def weights(n_in, n_out):
        Wm = np.zeros((n_out, n_in))
        for d in range(n_out):
            f = (d + 0.5) * n_in / n_out - 0.5
            s = math.floor(f)
            for k in range(-1, 3):
                Wm[d, min(max(s + k, 0), n_in - 1)] += keys(f - (s + k))
        return Wm
    for oh, ow in ((25, 31), (6, 5), (11, 29)):
        ref = weights(11, oh) @ x.astype(np.float64) @ weights(13, ow).T
        assert np.allclose(C.resize_cubic(x, oh, ow), ref, atol=2e-5 * np.abs(ref).max()), (oh, ow)
    assert np.array_equal(C.resize_cubic(x, 11, 13), x)


def test_bilateral_limits():
    # a constant map is returned as is
    z = np.full((10, 12), 0.5, np.float32)
    assert np.array_equal(C.bilateral(z), z)
    # a huge colour sigma makes it a normalised spatial Gaussian over the disc (centre weight 1), REFLECT_101 borders
    rng = np.random.default_rng(4)
    x = rng.uniform(0, 1, (9, 11)).astype(np.float32)
    out = C.bilateral(x, d=5, sigma_color=1e6, sigma_space=2.0)
    pad = np.pad(x.astype(np.float64), 2, mode="reflect")
    ref = np.zeros_like(x, dtype=np.float64)
    wsum = 0.0
    for i in range(-2, 3):
        for j in range(-2, 3):
            r = math.sqrt(i * i + j * j)
            if r > 2:
                continue
            w = math.exp(-r * r / 8.0)
            ref += w * pad[2 + i:2 + i + 9, 2 + j:2 + j + 11]
            wsum += w
    assert np.allclose(out, ref / wsum, rtol=2e-6, atol=1e-7)
    # a small colour sigma keeps a step edge: pixels far from the edge keep their side's value
    step = np.zeros((12, 12), np.float32)
    step[:, 6:] = 1.0
    out = C.bilateral(step, d=9, sigma_color=0.05, sigma_space=75.0)
    assert np.all(np.abs(out[:, :6]) < 1e-6) and np.all(np.abs(out[:, 6:] - 1.0) < 1e-6)
