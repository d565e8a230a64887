"""Sample workers of the input pipeline (imageselect_Dataloader_optflow.DataLoader(decode_procs=N)).

PIL's JPEG decode keeps the GIL for most of its run (measured here: 1 thread 546 images/s, 2 threads 938, 8
threads 903 for 192x512 strips), so N worker processes load whole samples instead -- the image decoded and the
raw label read straight into the loader's shared-memory staging area, the camera / projection files parsed
(8 processes: 3529 images/s on the same 8 cores).  This module imports only NumPy and PIL: the workers are
spawned fresh and never touch the GPU."""
from multiprocessing import shared_memory

import numpy as np

_attached = {}


def decode_into(shm_name, off, cap, path):
    """decode_jpeg (3 channels) of `path` into shared memory `shm_name` at byte `off` if it fits `cap` bytes.
    Returns (h, w, None) or, if it does not fit, (h, w, the decoded array)."""
    from PIL import Image
    sh = _attached.get(shm_name)
    if sh is None:
        sh = _attached[shm_name] = shared_memory.SharedMemory(name=shm_name)
        try:    # the loader owns (and unlinks) the segment; keep this process's tracker out of it
            from multiprocessing import resource_tracker
            resource_tracker.unregister(sh._name, "shared_memory")
        except Exception:
            pass
    with Image.open(path) as im:
        if im.mode != "RGB":
            im = im.convert("RGB")
        a = np.asarray(im, dtype=np.uint8)
    if a.nbytes > cap:
        return a.shape[0], a.shape[1], a
    np.ndarray((a.nbytes,), np.uint8, sh.buf, off)[:] = a.reshape(-1)
    return a.shape[0], a.shape[1], None


def csv_record(text, n, delim):
    """tf.decode_csv of one record of n float fields with record_defaults [[1.]] * n (empty field -> 1.0);
    the record is the file's content without its line terminator (imageselect_Dataloader_optflow.py:158-176)."""
    fields = text.rstrip("\r\n").split(delim)
    if len(fields) != n:
        raise ValueError(f"expected {n} '{delim}'-separated fields, got {len(fields)}")
    return np.array([float(v) if v.strip() else 1.0 for v in fields], dtype=np.float32)


def read_cam_proj(cam_path, proj_path):
    """(intrinsics [3,3], tgt2src_projs [2,4,4], m_scale) of one sample (:158-181)."""
    with open(cam_path) as fh:
        cam = csv_record(fh.read(), 9, ",").reshape(3, 3)
    with open(proj_path) as fh:
        pv = csv_record(fh.read(), 34, " ")[:-1]
    return cam, pv[:-1].reshape(2, 4, 4), pv[-1]


def load_sample(shm_name, off, cap, img_path, lab_off, lab_count, lab_path, cam_path, proj_path, drop=()):
    """One sample: the image into the segment at `off` (if it fits `cap` bytes), the raw float32 label
    (lab_count values) at `lab_off`, and the parsed camera / projection files.  `drop`: segments the loader
    has unlinked (a slot outgrew them); this worker closes its handles on them first.
    Returns (h, w, the image if it did not fit else None, cam, projs, m_scale)."""
    if drop:
        detach(drop)
    h, w, big = decode_into(shm_name, off, cap, img_path)
    v = np.fromfile(lab_path, dtype="<f4")
    if v.size != lab_count:
        raise ValueError(f"{lab_path}: {v.size} floats, expected {lab_count}")
    np.ndarray((lab_count,), np.float32, _attached[shm_name].buf, lab_off)[:] = v
    cam, projs, m = read_cam_proj(cam_path, proj_path)
    return h, w, big, cam, projs, m


def detach(names):
    """Drop this worker's handles on the given segments (the loader unlinks them)."""
    for n in names:
        sh = _attached.pop(n, None)
        if sh is not None:
            sh.close()
