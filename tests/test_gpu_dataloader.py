"""Input pipeline on the GPU: tde_image_resize_unpack bit-exact against the float32
restatement (oracle/dataloader.py) on ragged batches, up / down / identity scales, 1-3 frames and
channel-view outputs; the whole DataLoader (PIL decode -> pinned staging -> H2D -> one resize launch)
against oracle.load_batch for the same samples, epoch / last-partial-batch behaviour, shuffling, and a
config-2 training step fed from it."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import dataloader as OD
from tests.dataset_util import make_dataset

pytestmark = pytest.mark.gpu


def _resize_unpack(imgs, out_h, out_w, nframes, cstride=3, coff=0):
    from tf_depth_estimation_amd import _lib
    B = len(imgs)
    hdr = (16 * B + 255) // 256 * 256
    offs, off = [], hdr
    for a in imgs:
        offs.append(off)
        off += (a.nbytes + 15) // 16 * 16
    buf = np.zeros(off, np.uint8)
    buf[:8 * B] = np.array(offs, np.int64).view(np.uint8)
    buf[8 * B:16 * B] = np.array([[a.shape[0], a.shape[1]] for a in imgs], np.int32).reshape(-1).view(np.uint8)
    for o, a in zip(offs, imgs):
        buf[o:o + a.nbytes] = a.reshape(-1)
    dev = torch.from_numpy(buf).cuda()
    outs = [torch.full((B, out_h, out_w, cstride), -7.0, device="cuda") for _ in range(nframes)]
    a = _lib.ImageBatch()
    a.B, a.out_h, a.out_w, a.nframes = B, out_h, out_w, nframes
    a.src, a.src_off, a.src_hw = dev.data_ptr(), dev.data_ptr(), dev.data_ptr() + 8 * B
    for f in range(nframes):
        a.out[f], a.out_cstride[f], a.out_coff[f] = outs[f].data_ptr(), cstride, coff
    _lib.call("tde_image_resize_unpack", ctypes.byref(a), _lib.stream_ptr())
    torch.cuda.synchronize()
    return [o.cpu().numpy() for o in outs]


@pytest.mark.parametrize("sizes,out_h,out_w,nframes,cs,co", [
    ([(60, 180)], 60, 90, 2, 3, 0),                       # identity-size strip, 2 frames
    ([(61, 183), (30, 90), (90, 250)], 24, 36, 2, 3, 0),   # ragged batch, down and up
    ([(17, 29), (5, 7)], 40, 33, 1, 4, 1),                 # upsample, 1 frame into a channel view
    ([(48, 150), (48, 150)], 48, 50, 3, 4, 0),             # 3 frames, padded view
])
def test_resize_unpack_bit_exact(sizes, out_h, out_w, nframes, cs, co):
    rng = np.random.default_rng(sum(h * w for h, w in sizes))
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]
    got = _resize_unpack(imgs, out_h, out_w, nframes, cs, co)
    for b, img in enumerate(imgs):
        ref = OD.resize_bilinear_tf1(img, out_h, out_w * nframes)
        for f in range(nframes):
            np.testing.assert_array_equal(got[f][b, :, :, co:co + 3], ref[:, f * out_w:(f + 1) * out_w])
        if cs > 3:   # channels outside the view untouched
            keep = [c for c in range(cs) if not co <= c < co + 3]
            assert np.all(got[0][b][..., keep] == -7.0)


def test_resize_unpack_rejects_bad_arguments():
    from tf_depth_estimation_amd import _lib
    lib = _lib.load()
    a = _lib.ImageBatch()
    a.B, a.out_h, a.out_w, a.nframes = 1, 4, 4, 5
    assert lib.tde_image_resize_unpack(ctypes.byref(a), None) != 0
    a.nframes = 1
    assert lib.tde_image_resize_unpack(ctypes.byref(a), None) != 0     # null source


def _check_batch(got, fl, idx, ih, iw, ns, rh, rw):
    ref = OD.load_batch(fl, idx, ih, iw, ns, resized_h=rh, resized_w=rw)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g.cpu().numpy(), r)


@pytest.mark.parametrize("procs", [0, 2], ids=["threads", "procs"])
def test_loader_matches_oracle_in_order(tmp_path, procs):
    """procs=2: JPEG decode in two worker processes into shared memory (the 7th image is larger than the
    first: the slot's staging grows, in the shared segment too)."""
    import os
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader
    root = make_dataset(str(tmp_path), 7, sizes=[(60, 180)] * 6 + [(64, 200)])
    fl = OD.read_labeled_image_list(root, "train")
    shm_before = set(os.listdir("/dev/shm")) if os.path.isdir("/dev/shm") else set()
    dl = DataLoader(root, 3, 30, 90, 2, 4, "train", resizedheight=30, resizedwidth=90, shuffle=False,
                    num_epochs=2, workers=4, prefetch=2, decode_procs=procs)
    seen = []
    try:
        while True:
            batch = dl.load_train_batch()
            torch.cuda.synchronize()
            _check_batch(batch, fl, dl.last_indices, 30, 90, 4, 30, 90)
            seen.extend(dl.last_indices)
    except StopIteration:
        pass
    finally:
        dl.close()
    # 2 epochs x 7 samples in file order, batches of 3 across the epoch boundary, last partial batch dropped
    assert seen == ([0, 1, 2, 3, 4, 5, 6] * 2)[:12]
    if os.path.isdir("/dev/shm"):        # every shared staging segment unlinked by close()
        assert set(os.listdir("/dev/shm")) - shm_before == set()


def test_loader_shuffles_per_epoch(tmp_path):
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader
    root = make_dataset(str(tmp_path), 8)
    fl = OD.read_labeled_image_list(root, "train")
    dl = DataLoader(root, 4, 30, 90, 2, 4, "train", resizedheight=24, resizedwidth=72, num_epochs=3, seed=5,
                    workers=3)
    epochs = []
    try:
        for _ in range(6):
            batch = dl.load_train_batch()
            torch.cuda.synchronize()
            _check_batch(batch, fl, dl.last_indices, 30, 90, 4, 24, 72)
            epochs.append(list(dl.last_indices))
    finally:
        dl.close()
    e = [epochs[0] + epochs[1], epochs[2] + epochs[3], epochs[4] + epochs[5]]
    assert all(sorted(x) == list(range(8)) for x in e)      # each epoch is a permutation
    assert e[0] != e[1] or e[1] != e[2]


def test_loader_buffers_not_overwritten_while_held(tmp_path):
    """A batch stays intact until the consumer asks for the next one, even with every prefetch slot busy."""
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader
    root = make_dataset(str(tmp_path), 6)
    fl = OD.read_labeled_image_list(root, "train")
    dl = DataLoader(root, 2, 30, 90, 2, 4, "train", resizedheight=30, resizedwidth=90, shuffle=False,
                    num_epochs=4, prefetch=1)
    try:
        batch = dl.load_train_batch()
        idx = list(dl.last_indices)
        import time
        time.sleep(1.0)        # producer fills every free slot meanwhile
        torch.cuda.synchronize()
        _check_batch(batch, fl, idx, 30, 90, 4, 30, 90)
    finally:
        dl.close()


def test_loader_feeds_a_training_step(tmp_path):
    """train_depth_only.py:77-108 wiring: the loader's tgt image and label drive a config-2 step (images at
    the trainer's resolution, label at image_height x image_width)."""
    from tf_depth_estimation_amd import _api, train, variables
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader
    root = make_dataset(str(tmp_path), 4, strip_hw=(64, 192), image_hw=(64, 96))
    dl = DataLoader(root, 2, 64, 96, 2, 4, "train", resizedheight=64, resizedwidth=96, shuffle=False)
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    tr = train.DepthOnlyTrainer(2, 64, 96)
    try:
        for _ in range(2):
            tgt, src, label, intr, projs, m = dl.load_train_batch()
            tr.set_batch(tgt / 255.0 - 0.5, label)
            tr.step_eager()
        torch.cuda.synchronize()
        assert np.isfinite(tr.total_loss())
    finally:
        dl.close()


def _pose_vec(T):
    """[B,4,4] rigid motions -> [B,6] (translation, angle-axis rotation): the gt_right_cam layout of
    train_depth_then_cam_lr.py:117-118 (concat(translation, rotation))."""
    from scipy.spatial.transform import Rotation
    T = np.asarray(T, np.float64)
    return np.concatenate([T[:, :3, 3], Rotation.from_matrix(T[:, :3, :3]).as_rotvec()], 1).astype(np.float32)


def test_loader_feeds_a_config4_step(tmp_path):
    """config 4 (train_depth_then_cam_lr.py:117-154 wiring, with the imageselect loader the
    script has commented in at :104-115) trained from the built loader: tgt -> image_left, src -> image_right (both
    /255 - 0.5), the label, the loader's multi-scale intrinsics, and the camera from the first tgt2src projection
    (a rigid motion -> (t, angle-axis)).  The first step's loss terms equal the float64 oracle's on the same batch
    (1e-5; consistency 1e-4), and captured steps on the next batches stay finite."""
    from oracle import losses as OL
    from oracle import nets as ON
    from test_gpu_nets import oracle_params_from
    from tf_depth_estimation_amd import _api, train, variables
    from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader
    B, H, W = 2, 64, 96
    root = make_dataset(str(tmp_path), 6, strip_hw=(64, 192), image_hw=(H, W), rigid=True)
    dl = DataLoader(root, B, H, W, 1, 4, "train", resizedheight=H, resizedwidth=W, shuffle=False, num_epochs=2)
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    tr = train.DepthThenCamTrainer(B, H, W)
    try:
        tgt, src, label, intr, projs, m = dl.load_train_batch()
        il, ir = tgt / 255.0 - 0.5, src[..., :3] / 255.0 - 0.5
        gt = torch.from_numpy(_pose_vec(projs[:, 0].cpu().numpy())).cuda()
        assert intr.shape == (B, 4, 3, 3) and projs.shape == (B, 2, 4, 4)
        tr.set_batch(il, ir, label, intr, gt)
        P = {dt: (oracle_params_from(tr.single.chunk, "", dt), oracle_params_from(tr.pair.chunk, "", dt))
             for dt in (torch.float64,)}
        tr.phase_compute()
        torch.cuda.synchronize()
        parts = tr.loss_parts()
        Pss, Ppp = P[torch.float64]
        x = {k: v.detach().double().cpu() for k, v in dict(il=il, ir=ir).items()}
        dsl = ON.disp_net(Pss, x["il"], True, scope="model_singledepth/depth_net")
        dsr = ON.disp_net(Pss, x["ir"], True, scope="model_singledepth/depth_net")
        dpl, pr, ml = ON.depth_net(Ppp, torch.cat([x["il"], x["ir"]], -1), True, scope="model_pairdepth/depth_cam_net",
                                   levels=4)
        dpr, pl, mr = ON.depth_net(Ppp, torch.cat([x["ir"], x["il"]], -1), True, scope="model_pairdepth/depth_cam_net",
                                   levels=4)
        total, rp = OL.loss_depth_then_cam_lr(dsl, dsr, dpl, dpr, pr, pl, ml, mr, x["il"], x["ir"],
                                              label.double().cpu(), intr.double().cpu(), gt.double().cpu())

        def val(t):
            return t.item() if torch.is_tensor(t) else float(t)
        for k in ("smooth", "depth", "exp", "cam"):
            assert abs(parts[k] - val(rp[k])) <= 1e-5 * abs(val(rp[k])) + 1e-9, (k, parts[k], val(rp[k]))
        assert abs(parts["photo"] - val(rp["pixel"])) <= 1e-5 * val(rp["pixel"]) + 1e-9
        assert abs(parts["consist"] - val(rp["consist"])) <= 1e-4 * val(rp["consist"]) + 1e-9
        tr.capture(warmup=1)
        for _ in range(2):
            tgt, src, label, intr, projs, m = dl.load_train_batch()
            tr.set_batch(tgt / 255.0 - 0.5, src[..., :3] / 255.0 - 0.5, label, intr,
                         torch.from_numpy(_pose_vec(projs[:, 0].cpu().numpy())).cuda())
            tr.step()
        torch.cuda.synchronize()
        assert np.isfinite(tr.total_loss())
        assert all(torch.isfinite(c.flat).all() for c in tr.chunks)
    finally:
        dl.close()
        tr.release_graphs()
        _api.clear_programs()
