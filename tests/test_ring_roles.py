"""CPU-side checks of the ring-tile role mask (tde_set_conv_ring, ABI 9) and the role-aware split-image op codes of
tde_conv2d_split_weights_size: which call reads which pre-split image is host logic, answered without a device.
(The GPU parity of the ring tiles themselves: tests/test_gpu_kernels.py::test_ring_presplit_weights.)"""
import ctypes

import pytest

from tf_depth_estimation_amd import _lib


def same_pad(n, k, s):
    out = (n + s - 1) // s
    pad = max((out - 1) * s + k - n, 0)
    return out, pad // 2


def conv_desc(N, H, W, C, K, k, s):
    d = _lib.ConvDesc()
    OH, pt = same_pad(H, k, s)
    OW, pl = same_pad(W, k, s)
    d.N, d.H, d.W, d.C, d.OH, d.OW, d.K, d.KH, d.KW = N, H, W, C, OH, OW, K, k, k
    d.stride, d.pad_top, d.pad_left, d.w_cin = s, pt, pl, C
    d.x_cstride, d.x_coff, d.y_cstride, d.y_coff = C, 0, K, 0
    return d


@pytest.fixture
def lib():
    lib = _lib.load()
    prev_math = lib.tde_get_conv_math()
    prev_ring = lib.tde_get_conv_ring()
    assert lib.tde_set_conv_math(4) == 0
    yield lib
    lib.tde_set_conv_math(prev_math)
    lib.tde_set_conv_ring(prev_ring)


def sizes(lib, d, deconv=False):
    return [lib.tde_conv2d_split_weights_size(ctypes.byref(d), o | (2 if deconv else 0)) for o in (0, 1)]


def test_set_conv_ring_range(lib):
    prev = lib.tde_set_conv_ring(7)
    assert 0 <= prev <= 15
    assert lib.tde_get_conv_ring() == 7
    assert lib.tde_set_conv_ring(16) == -1 and lib.tde_get_conv_ring() == 7
    assert lib.tde_set_conv_ring(-1) == -1
    assert lib.tde_set_conv_ring(0) == 7 and lib.tde_get_conv_ring() == 0


def test_conv_images_follow_the_call_role(lib):
    # icnv5-like (deep, stride 1, 64-row tiles): image 0 = the forward's, image 1 = the data gradient's
    d = conv_desc(16, 12, 16, 512, 256, 3, 1)
    lib.tde_set_conv_ring(0)
    assert sizes(lib, d) == [0, 0]
    lib.tde_set_conv_ring(1)                      # forward calls
    s = sizes(lib, d)
    assert s[0] > 0 and s[1] == 0
    lib.tde_set_conv_ring(2)                      # data-gradient calls
    s = sizes(lib, d)
    assert s[0] == 0 and s[1] > 0
    lib.tde_set_conv_ring(8)                      # deep forward calls: this layer's GEMM gets 64-row tiles
    s = sizes(lib, d)
    assert s[0] > 0 and s[1] == 0
    lib.tde_set_conv_ring(4)                      # filter gradients read no image
    assert sizes(lib, d) == [0, 0]


def test_deconv_images_follow_the_call_role(lib):
    # a deconv's virtual conv: its forward reads image 1 (op code 3), its data gradient image 0 (op code 2)
    d = conv_desc(16, 24, 32, 128, 256, 3, 2)     # virtual conv of a 12x16 -> 24x32 deconv, 256 -> 128 channels
    lib.tde_set_conv_ring(1)
    s = sizes(lib, d, deconv=True)
    assert s[0] == 0 and s[1] > 0
    lib.tde_set_conv_ring(2)
    s = sizes(lib, d, deconv=True)
    assert s[0] > 0 and s[1] == 0


def test_deep_mask_skips_128_row_tiles(lib):
    # a large-M strided layer (cnv2-like at twin batch 16: 128-row tiles) is on the ring for mask 1, not for mask 8
    d = conv_desc(16, 96, 128, 32, 64, 5, 2)
    lib.tde_set_conv_ring(1)
    assert sizes(lib, d)[0] > 0
    lib.tde_set_conv_ring(8)
    assert sizes(lib, d)[0] == 0


def test_halo_images_are_role_independent(lib):
    # a halo-path layer (stride 1, few channels, high resolution) keeps its split images whatever the ring mask
    d = conv_desc(16, 96, 128, 32, 32, 7, 1)
    lib.tde_set_conv_ring(0)
    s0 = sizes(lib, d)
    lib.tde_set_conv_ring(7)
    assert sizes(lib, d) == s0 and s0[0] > 0


def test_large_kernel_pixel_shuffle_takes_no_ring_image(lib):
    # a 5x5 / 7x7 stride-2 deconv large enough for the pixel-shuffle GEMM runs its register-staged form (the ring's
    # B-image prep gathers the 3x3 form only): no split image for its forward, whatever the ring mask
    for k in (5, 7):
        d = conv_desc(16, 128, 96, 16, 32, k, 2)   # virtual conv of a 64x48 -> 128x96 deconv, 32 -> 16 channels
        lib.tde_set_conv_ring(7)
        s = sizes(lib, d, deconv=True)
        assert s[1] == 0, (k, s)
