"""imageselect_Dataloader_optflow.DataLoader restated in NumPy (TEST INFRASTRUCTURE ONLY; see
oracle/__init__.py): the file list, the per-file parsing, TF-1's bilinear resize_images in float32 and the
sequence unpacking, the batch assembly and the multi-scale intrinsics -- the checker of
tf_depth_estimation_amd.imageselect_Dataloader_optflow (host pipeline + tde_image_resize_unpack).

JPEG decoding is PIL's (libjpeg, ISLOW IDCT, fancy chroma upsampling), the same decoder the product's host
half uses; TF's decode_jpeg (libjpeg-turbo, dct_method "" = ISLOW) is not importable here, so against TF
the decoded pixels are parity unpinned.  Everything after the decode is pinned by the
known-answer tests in tests/test_dataloader.py.
"""
import os

import numpy as np

RESIZED_H, RESIZED_W = 240, 720      # imageselect_Dataloader_optflow.py:24-25


def read_labeled_image_list(dataset_dir, split):
    """imageselect_Dataloader_optflow.py:66-101: '<subfolder> <a> <b>' lines of <split>.txt ->
    <sub>/<a>_<b>.jpg, <sub>/<a>_<b>_cam.txt, <sub>/frame<a>_<b>.jpg_z.bin, <sub>/<a>_<b>_tgt2src_proj.txt.
    The frame id drops the line's last character (x.split(' ')[2][:-1]: the newline)."""
    with open(os.path.join(dataset_dir, "%s.txt" % split)) as f:
        frames = f.readlines()
    subfolders = [x.split(" ")[0] for x in frames]
    frame_ids = [x.split(" ")[1] + "_" + x.split(" ")[2][:-1] for x in frames]
    j = os.path.join
    return {
        "image_file_list": [j(dataset_dir, subfolders[i], frame_ids[i] + ".jpg") for i in range(len(frames))],
        "cam_file_list": [j(dataset_dir, subfolders[i], frame_ids[i] + "_cam.txt") for i in range(len(frames))],
        "gt_depth_file_list": [j(dataset_dir, subfolders[i], "frame" + frame_ids[i] + ".jpg" + "_z.bin")
                               for i in range(len(frames))],
        "tgt2src_proj_list": [j(dataset_dir, subfolders[i], frame_ids[i] + "_tgt2src_proj.txt")
                              for i in range(len(frames))],
    }


def decode_csv_record(text, n, delim=","):
    """tf.decode_csv of ONE record with n float fields, record_defaults [[1.]] * n: an empty field takes
    the default 1.0 (imageselect_Dataloader_optflow.py:159-166,171-176).  The record is the whole file
    minus its line terminator."""
    rec = text.rstrip("\r\n")
    fields = rec.split(delim)
    if len(fields) != n:
        raise ValueError(f"expected {n} fields, got {len(fields)}")
    return np.array([float(v) if v.strip() != "" else 1.0 for v in fields], dtype=np.float32)


def read_cam(path):
    """intrinsics = reshape(decode_csv(cam_file, 9 x [1.]), [3, 3]) (:158-166)."""
    with open(path) as f:
        return decode_csv_record(f.read(), 9).reshape(3, 3)


def read_proj(path):
    """:171-181: 34 space-delimited fields; drop the last; m_scale = the new last; the first 32 -> [2,4,4]."""
    with open(path) as f:
        v = decode_csv_record(f.read(), 34, " ")[:-1]
    return v[:-1].reshape(2, 4, 4), np.float32(v[-1])


def read_label(path, image_height, image_width):
    """label = reshape(decode_raw(label_file, float32), [image_height, image_width, 1]) (:138-144)."""
    return np.fromfile(path, dtype="<f4").reshape(image_height, image_width, 1)


def decode_jpeg(path):
    """decode_jpeg (3 channels, uint8 HWC) -- PIL's libjpeg decode (see the module note)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def resize_bilinear_tf1(img, out_h, out_w):
    """tf.image.resize_images default (ResizeMethod.BILINEAR, align_corners=False) in TF-1's float32
    arithmetic (resize_bilinear_op.cc): scale = in / (float)out; in = i * scale; lower = (int)in;
    upper = min(lower + 1, in - 1); lerp = in - lower; top = tl + (tr - tl) * xl, bottom likewise,
    out = top + (bottom - top) * yl, each operation rounded to float32 (no fused multiply-add)."""
    h, w, c = img.shape
    f = np.float32
    sy, sx = f(f(h) / f(out_h)), f(f(w) / f(out_w))
    iny = (np.arange(out_h, dtype=np.float32) * sy).astype(np.float32)
    inx = (np.arange(out_w, dtype=np.float32) * sx).astype(np.float32)
    y0 = iny.astype(np.int64)
    x0 = inx.astype(np.int64)
    y1 = np.minimum(y0 + 1, h - 1)
    x1 = np.minimum(x0 + 1, w - 1)
    ly = (iny - y0.astype(np.float32)).astype(np.float32)[:, None, None]
    lx = (inx - x0.astype(np.float32)).astype(np.float32)[None, :, None]
    im = img.astype(np.float32)
    tl, tr = im[y0][:, x0], im[y0][:, x1]
    bl, br = im[y1][:, x0], im[y1][:, x1]
    top = (tl + ((tr - tl).astype(f) * lx).astype(f)).astype(f)
    bot = (bl + ((br - bl).astype(f) * lx).astype(f)).astype(f)
    return (top + ((bot - top).astype(f) * ly).astype(f)).astype(f)


def unpack_image_sequence(image_seq, image_width):
    """:216-233: tgt = columns [0, W), src_image_1 = columns [W, 2W)."""
    return image_seq[:, :image_width], image_seq[:, image_width:2 * image_width]


def make_intrinsics_matrix(fx, fy, cx, cy):
    """:236-246 ([B] each -> [B,3,3])."""
    B = fx.shape[0]
    z = np.zeros(B, np.float32)
    r1 = np.stack([fx, z, cx], axis=1)
    r2 = np.stack([z, fy, cy], axis=1)
    r3 = np.tile(np.array([[0.0, 0.0, 1.0]], np.float32), (B, 1))
    return np.stack([r1, r2, r3], axis=1).astype(np.float32)


def get_multi_scale_intrinsics(intrinsics, num_scales, x_resize_ratio, y_resize_ratio):
    """:248-262: per scale s, f/(2**s)*ratio and c/(2**s)*ratio in float32 -> [B, num_scales, 3, 3]."""
    f = np.float32
    out = []
    for s in range(num_scales):
        d = f(2 ** s)
        fx = ((intrinsics[:, 0, 0] / d).astype(f) * f(x_resize_ratio)).astype(f)
        fy = ((intrinsics[:, 1, 1] / d).astype(f) * f(y_resize_ratio)).astype(f)
        cx = ((intrinsics[:, 0, 2] / d).astype(f) * f(x_resize_ratio)).astype(f)
        cy = ((intrinsics[:, 1, 2] / d).astype(f) * f(y_resize_ratio)).astype(f)
        out.append(make_intrinsics_matrix(fx, fy, cx, cy))
    return np.stack(out, axis=1)


def load_batch(files, indices, image_height, image_width, num_scales, resized_h=RESIZED_H, resized_w=RESIZED_W):
    """One batch of load_train_batch (:28-63) for the given sample indices, in order:
    (tgt_image, src_image_stack, label, intrinsics [B,num_scales,3,3], tgt2src_projs [B,2,4,4], m_scale [B])."""
    tgts, srcs, labels, cams, projs, ms = [], [], [], [], [], []
    for i in indices:
        seq = resize_bilinear_tf1(decode_jpeg(files["image_file_list"][i]), resized_h, resized_w * 2)
        t, s = unpack_image_sequence(seq, resized_w)
        tgts.append(t)
        srcs.append(s)
        labels.append(read_label(files["gt_depth_file_list"][i], image_height, image_width))
        cams.append(read_cam(files["cam_file_list"][i]))
        p, m = read_proj(files["tgt2src_proj_list"][i])
        projs.append(p)
        ms.append(m)
    # x / y resize ratio: tf.cast(resizedwidth, float32) / image_width (:59-60)
    xr = np.float32(np.float32(resized_w) / np.float32(image_width))
    yr = np.float32(np.float32(resized_h) / np.float32(image_height))
    intr = get_multi_scale_intrinsics(np.stack(cams), num_scales, xr, yr)
    return (np.stack(tgts), np.stack(srcs), np.stack(labels), intr, np.stack(projs), np.array(ms, np.float32))
