"""Input pipeline (imageselect_Dataloader_optflow.py): CPU checks of the oracle's
restatement (known answers of TF-1's resize_images, decode_csv defaults, proj / cam / label parsing,
multi-scale intrinsics) and of the product loader's host logic against it.  The device half
(tde_image_resize_unpack) and the whole pipeline run in tests/test_gpu_dataloader.py."""
import os

import numpy as np
import pytest

from oracle import dataloader as OD
from tests.dataset_util import make_dataset


def test_resize_identity_is_exact():
    img = np.random.default_rng(0).integers(0, 256, (7, 9, 3), dtype=np.uint8)
    assert np.array_equal(OD.resize_bilinear_tf1(img, 7, 9), img.astype(np.float32))


def test_resize_upsample_known_answer():
    # 1x2 -> 1x4: src x = 0, 0.5, 1, 1.5 -> [a, (a+b)/2, b, b] (upper clamped to the last column)
    img = np.array([[[10, 20, 30], [50, 60, 70]]], np.uint8)
    out = OD.resize_bilinear_tf1(img, 1, 4)
    np.testing.assert_array_equal(out[0, :, 0], [10, 30, 50, 50])
    np.testing.assert_array_equal(out[0, :, 2], [30, 50, 70, 70])


def test_resize_downsample_by_two_picks_even_pixels():
    img = np.random.default_rng(1).integers(0, 256, (8, 12, 3), dtype=np.uint8)
    out = OD.resize_bilinear_tf1(img, 4, 6)
    np.testing.assert_array_equal(out, img[::2, ::2].astype(np.float32))


def test_resize_matches_float64_formula():
    img = np.random.default_rng(2).integers(0, 256, (11, 17, 3), dtype=np.uint8)
    out = OD.resize_bilinear_tf1(img, 7, 40)
    f = img.astype(np.float64)
    ref = np.zeros((7, 40, 3))
    for y in range(7):
        iy = y * np.float32(11 / np.float32(7))
        y0 = int(iy); y1 = min(y0 + 1, 10); ly = iy - y0
        for x in range(40):
            ix = x * np.float32(17 / np.float32(40))
            x0 = int(ix); x1 = min(x0 + 1, 16); lx = ix - x0
            top = f[y0, x0] + (f[y0, x1] - f[y0, x0]) * lx
            bot = f[y1, x0] + (f[y1, x1] - f[y1, x0]) * lx
            ref[y, x] = top + (bot - top) * ly
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-4)


def test_decode_csv_defaults_and_field_count():
    np.testing.assert_array_equal(OD.decode_csv_record("1,,3\n", 3), [1, 1, 3])
    with pytest.raises(ValueError):
        OD.decode_csv_record("1,2", 3)


def test_proj_parsing_drops_the_trailing_field(tmp_path):
    v = np.arange(33, dtype=np.float32) * 0.5
    p = tmp_path / "p.txt"
    p.write_text(" ".join(str(x) for x in v) + " ")
    projs, m = OD.read_proj(str(p))
    np.testing.assert_array_equal(projs.reshape(-1), v[:32])
    assert m == v[32]


def test_multi_scale_intrinsics_known_answer():
    K = np.array([[[100.0, 0, 40.0], [0, 80.0, 30.0], [0, 0, 1]]], np.float32)
    out = OD.get_multi_scale_intrinsics(K, 3, 2.0, 0.5)
    assert out.shape == (1, 3, 3, 3)
    np.testing.assert_array_equal(out[0, 0], [[200, 0, 80], [0, 40, 15], [0, 0, 1]])
    np.testing.assert_array_equal(out[0, 2], [[50, 0, 20], [0, 10, 3.75], [0, 0, 1]])


def test_file_list_layout(tmp_path):
    root = make_dataset(str(tmp_path), 4)
    fl = OD.read_labeled_image_list(root, "train")
    assert fl["image_file_list"][1] == os.path.join(root, "seq1", "0001_07.jpg")
    assert fl["gt_depth_file_list"][1] == os.path.join(root, "seq1", "frame0001_07.jpg_z.bin")
    assert fl["cam_file_list"][0].endswith("seq0/0000_00_cam.txt")
    assert fl["tgt2src_proj_list"][0].endswith("seq0/0000_00_tgt2src_proj.txt")
    for k in fl:
        assert all(os.path.exists(p) for p in fl[k])


def test_oracle_batch_shapes(tmp_path):
    root = make_dataset(str(tmp_path), 3)
    fl = OD.read_labeled_image_list(root, "train")
    tgt, src, lab, intr, projs, m = OD.load_batch(fl, [2, 0], 30, 90, 4, resized_h=24, resized_w=72)
    assert tgt.shape == (2, 24, 72, 3) and src.shape == (2, 24, 72, 3)
    assert lab.shape == (2, 30, 90, 1) and intr.shape == (2, 4, 3, 3)
    assert projs.shape == (2, 2, 4, 4) and m.shape == (2,)
    assert tgt.dtype == np.float32 and 0 <= tgt.min() and tgt.max() <= 255


def test_product_host_logic_matches_oracle(tmp_path):
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader, _csv_record
    root = make_dataset(str(tmp_path), 5)
    dl = DataLoader(root, 2, 30, 90, 2, 4, "train")
    assert dl.read_labeled_image_list() == OD.read_labeled_image_list(root, "train")
    K = np.random.default_rng(3).uniform(10, 300, (3, 3, 3)).astype(np.float32)
    np.testing.assert_array_equal(dl.get_multi_scale_intrinsics(K, 4, np.float32(8 / 3), np.float32(0.5)),
                                  OD.get_multi_scale_intrinsics(K, 4, np.float32(8 / 3), np.float32(0.5)))
    np.testing.assert_array_equal(_csv_record("1, 2,,4\n", 4, ","), OD.decode_csv_record("1, 2,,4\n", 4))


def _die(code):
    import os
    os._exit(code)


def test_dead_decode_worker_raises_not_hangs():
    """a decode worker that dies mid-task (OOM kill, decoder crash) must surface as an error in the
    loader instead of blocking the producer forever (multiprocessing.Pool replaces the worker but never
    completes its task)."""
    import multiprocessing as mp
    import threading
    import types
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader
    pool = mp.get_context("spawn").Pool(1)
    try:
        fake = types.SimpleNamespace(_task_timeout=60.0, _stop=threading.Event(), _worker_procs=list(pool._pool))
        fu = pool.apply_async(_die, (3,))
        with pytest.raises(RuntimeError, match="exited with code 3"):
            DataLoader._await(fake, fu)
        fake = types.SimpleNamespace(_task_timeout=0.5, _stop=threading.Event(), _worker_procs=[])
        import time
        fu = pool.apply_async(time.sleep, (5,))
        with pytest.raises(TimeoutError):
            DataLoader._await(fake, fu)
    finally:
        pool.terminate()
        pool.join()
