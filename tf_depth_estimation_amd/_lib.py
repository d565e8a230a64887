"""ctypes binding of libtde.so (the C ABI declared in include/tde.h).

The library is built in-tree by `make -C tf_depth_estimation_amd/csrc` (or __graft_entry__.build()).
It is loaded *after* torch so that its DT_NEEDED libamdhip64.so.7 resolves to the HIP runtime torch
already loaded (one runtime per process: torch's streams and allocations are valid in our calls).
There is no fallback: if the library is missing, `load()` raises.
"""
import ctypes
import gc
import os

import torch  # noqa: F401  (must be imported first, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtde.so")
ABI_VERSION = 10
BOUND_SLOTS = 16   # TDE_BOUND_SLOTS: an operand bound is the max of this many device floats
# tde_set_conv_math modes (include/tde.h): exact fp32 MFMA, bf16x3 (~2^-16 per product), and the
# fp32-accurate three-way bf16 split ("bf16x6": staged in LDS / split in registers)
CONV_MATH = {"fp32": 0, "bf16x3": 1, "bf16x6": 2, "bf16x6r": 3, "fp16x3": 4}

c_int, c_float, c_size_t, c_void_p, c_double_p = (ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_double))


class ConvDesc(ctypes.Structure):
    """Mirror of tde_conv_desc_t (include/tde.h)."""
    _fields_ = [(n, c_int) for n in ("N", "H", "W", "C", "OH", "OW", "K", "KH", "KW", "stride", "pad_top",
                                     "pad_left", "w_cin", "x_cstride", "x_coff", "y_cstride", "y_coff")] + \
               [("x_absmax", c_void_p), ("y_absmax", c_void_p), ("w_absmax", c_void_p), ("w_split", c_void_p * 2)]


P = c_void_p


class BnTrain(ctypes.Structure):
    """Mirror of tde_bn_train_t (include/tde.h): batch norm + ReLU fused behind a conv."""
    _fields_ = [("beta", P), ("eps", c_float), ("decay", c_float), ("bessel", c_int), ("moving_mean", P),
                ("moving_var", P), ("save_mean", P), ("save_invstd", P), ("y", P), ("y_cstride", c_int),
                ("y_coff", c_int), ("relu", c_int), ("groups", c_int), ("sums", P)]


class WarpLossArgs(ctypes.Structure):
    """Mirror of tde_warp_loss_t (include/tde.h)."""
    _fields_ = [("B", c_int), ("H", c_int), ("W", c_int),
                ("disp", P), ("disp_cs", c_int), ("disp_co", c_int),
                ("flow", P), ("flow_cs", c_int), ("flow_co", c_int),
                ("P", P), ("Kinv", P), ("img_src", P), ("img_tgt", P), ("wmask", P),
                ("logits", P), ("logit_cs", c_int), ("logit_co", c_int),
                ("disp_other", P), ("other_cs", c_int), ("other_co", c_int),
                ("photo_w", c_float), ("exp_w", c_float), ("consist_w", c_float),
                ("loss", P), ("g_disp", P), ("g_flow", P), ("g_logits", P), ("g_other", P), ("g_P", P),
                ("det_ws", P), ("det_ws_bytes", c_size_t)]


class PosePrepArgs(ctypes.Structure):
    """Mirror of tde_pose_prep_t (include/tde.h): one job of tde_pose_prep_multi."""
    _fields_ = [("B", c_int), ("pose_vec", P), ("pose_mat", P), ("K", P), ("T", P), ("P", P), ("Kinv", P)]


class PoseGradArgs(ctypes.Structure):
    """Mirror of tde_pose_grad_t (include/tde.h): one job of tde_pose_grad_spread."""
    _fields_ = [("B", c_int), ("nscales", c_int), ("pose_vec", P), ("K", P), ("k_stride_b", ctypes.c_long),
                ("gP", P), ("gT_extra", P), ("g_pose_vec", P), ("accumulate", c_int),
                ("dpose", P), ("hw", c_int), ("dpose_cstride", c_int), ("dpose_accumulate", c_int)]


WARP_MULTI_MAX = 8      # TDE_WARP_MULTI_MAX
PYR_MULTI_MAX = 4       # TDE_PYR_MULTI_MAX


class DepthLoss(ctypes.Structure):
    """Mirror of tde_depth_loss_t (include/tde.h): the multi-scale smooth + depth-L1 loss head."""
    _fields_ = [("N", c_int), ("H", c_int), ("W", c_int), ("nscales", c_int),
                ("pred", P * 4), ("pred_cs", c_int * 4), ("pred_co", c_int * 4),
                ("grad", P * 4), ("g_cs", c_int * 4), ("g_co", c_int * 4),
                ("smooth_w", c_float * 4), ("recip", c_int), ("label", P), ("nonfinite", c_int),
                ("l1_w", c_float * 4), ("loss_smooth", P), ("loss_l1", P), ("grad_accumulate", c_int)]


class ImageBatch(ctypes.Structure):
    """Mirror of tde_image_batch_t (include/tde.h): the input pipeline's resize + unpack launch."""
    _fields_ = [("B", c_int), ("out_h", c_int), ("out_w", c_int), ("nframes", c_int),
                ("src", P), ("src_off", P), ("src_hw", P),
                ("out", P * 4), ("out_cstride", c_int * 4), ("out_coff", c_int * 4)]


_SIGS = {
    "tde_conv2d_split_weights_size": (c_size_t, [P, c_int]),
    "tde_conv2d_split_weights": (c_int, [c_int, P, P, P, P, P]),
    "tde_image_resize_unpack": (c_int, [P, P]),
    "tde_resize_area_u8": (c_int, [c_int, c_int, c_int, c_int, P, c_int, c_int, P, P, c_int, P]),
    "tde_resize_cubic_f32": (c_int, [c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "tde_bilateral_workspace_size": (c_size_t, [c_int]),
    "tde_bilateral_f32": (c_int, [c_int, c_int, c_int, P, P, c_int, ctypes.c_double, ctypes.c_double, P, c_size_t,
                                  P]),
    "tde_loss_depth_pyramid": (c_int, [P, P]),
    "tde_warp_loss_multi": (c_int, [P, c_int, P]),
    "tde_loss_depth_pyramid_multi": (c_int, [P, c_int, P]),
    "tde_pose_prep_multi": (c_int, [P, c_int, P]),
    "tde_pose_grad_spread": (c_int, [P, c_int, P]),
    "tde_warp_loss": (c_int, [P, P]),
    "tde_warp_loss_det_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "tde_warp_fwd": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, P, P, P, c_int, c_int, P, P, P, P, P, P, P]),
    "tde_pose_prep": (c_int, [c_int, P, P, P, P, P, P, P]),
    "tde_pose_grad": (c_int, [c_int, c_int, P, P, ctypes.c_long, P, P, P, c_int, P]),
    "tde_cam_loss": (c_int, [c_int, P, P, P, c_float, P, P, P, P]),
    "tde_pose_vec2mat": (c_int, [c_int, P, c_int, P, P]),
    "tde_pose_vec2mat_bwd": (c_int, [c_int, P, c_int, P, P, c_int, P]),
    "tde_sampler_bwd": (c_int, [c_int, c_int, c_int, c_int, P, P, c_int, c_int, P, P, P, P, P]),
    "tde_cam_coords_bwd": (c_int, [c_int, c_int, c_int, P, P, P, P, P, P, c_int, P, P]),
    "tde_pose_dp_to_dt": (c_int, [c_int, P, P, P, P]),
    "tde_abi_version": (c_int, []),
    "tde_crc32c": (ctypes.c_uint32, [P, c_size_t, ctypes.c_uint32]),
    "tde_status_string": (ctypes.c_char_p, [c_int]),
    "tde_set_conv_math": (c_int, [c_int]),
    "tde_get_conv_math": (c_int, []),
    "tde_conv_span_arm": (c_int, [P, P]),
    "tde_stamp": (c_int, [P, P]),
    "tde_conv2d_workspace_size": (c_size_t, [P, c_int]),
    "tde_deconv2d_workspace_size": (c_size_t, [P, c_int]),
    "tde_conv2d_fwd": (c_int, [P, P, P, P, c_int, P, c_size_t, P]),
    "tde_conv2d_fwd_bn": (c_int, [P, P, P, P, P, P, c_size_t, P]),
    "tde_deconv2d_fwd_bn": (c_int, [P, P, P, P, P, P, c_size_t, P]),
    "tde_conv2d_fwd_bias_act": (c_int, [P, P, P, P, c_int, P, P, c_size_t, P]),
    "tde_deconv2d_fwd_bias_act": (c_int, [P, P, P, P, c_int, P, P, c_size_t, P]),
    "tde_bn_fold": (c_int, [c_int, c_int, c_int, c_int, P, P, P, P, c_float, P, P, P]),
    "tde_conv2d_bwd_workspace_size": (c_size_t, [P]),
    "tde_deconv2d_bwd_workspace_size": (c_size_t, [P]),
    "tde_conv2d_bwd": (c_int, [P, P, P, P, P, c_int, P, c_int, P, c_size_t, P]),
    "tde_deconv2d_bwd": (c_int, [P, P, P, P, P, c_int, P, c_int, P, c_size_t, P]),
    "tde_conv2d_bwd_data": (c_int, [P, P, P, P, c_int, P, c_size_t, P]),
    "tde_conv2d_bwd_filter": (c_int, [P, P, P, P, c_int, P, c_size_t, P]),
    "tde_deconv2d_fwd": (c_int, [P, P, P, P, c_int, P, c_size_t, P]),
    "tde_deconv2d_bwd_data": (c_int, [P, P, P, P, c_int, P, c_size_t, P]),
    "tde_deconv2d_bwd_filter": (c_int, [P, P, P, P, c_int, P, c_size_t, P]),
    "tde_head_workspace_size": (c_size_t, [P]),
    "tde_head_fwd": (c_int, [P, P, P, P, P, c_int, c_float, c_float, P]),
    "tde_head_bwd": (c_int, [P, P, P, P, P, P, c_int, P, P, c_int, c_int, c_float, c_float, P, c_size_t, P]),
    "tde_bn_workspace_size": (c_size_t, [c_int, c_int]),
    "tde_bn_fwd_train": (c_int, [c_int, c_int, c_int, P, P, c_float, c_float, c_int, P, P, P, P, P, c_int, c_int,
                                 c_int, P, c_size_t, P]),
    "tde_bn_fwd_infer": (c_int, [c_int, c_int, P, P, c_float, P, P, P, c_int, c_int, c_int, P]),
    "tde_bn_bwd": (c_int, [c_int, c_int, c_int, P, P, P, P, P, c_int, c_int, P, P, c_int, c_int, P, P, c_size_t,
                           P]),
    "tde_bias_relu_bwd": (c_int, [c_int, c_int, P, c_int, c_int, P, c_int, c_int, c_int, P, P, c_int, P, P, c_size_t,
                                  P]),
    "tde_bn_sums": (c_int, [c_int, c_int, c_int, P, P, c_int, c_int, P, P, P, c_int, c_int, P, P, P, c_size_t, P]),
    "tde_bn_fwd_from_sums": (c_int, [c_int, c_int, c_int, ctypes.c_long, P, P, P, c_float, c_float, c_int, P, P, P,
                                     P, P, c_int, c_int, c_int, P]),
    "tde_bn_bwd_from_sums": (c_int, [c_int, c_int, c_int, ctypes.c_long, P, P, P, P, P, c_int, c_int, P, P, P, P,
                                     c_int, c_int, P, P]),
    "tde_resize_nearest_fwd": (c_int, [c_int] * 4 + [P, c_int, c_int, c_int, c_int, P, c_int, c_int, P]),
    "tde_resize_nearest_bwd": (c_int, [c_int] * 4 + [P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P]),
    "tde_resize_bilinear_fwd": (c_int, [c_int] * 4 + [P, c_int, c_int, c_int, c_int, P, c_int, c_int, P]),
    "tde_resize_bilinear_bwd": (c_int, [c_int] * 4 + [P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P]),
    "tde_resize_area_fwd": (c_int, [c_int] * 4 + [P, c_int, c_int, P, P]),
    "tde_loss_smooth2": (c_int, [c_int, c_int, c_int, P, c_int, c_int, c_int, c_float, P, P, c_int, c_int, P]),
    "tde_loss_sig_l2": (c_int, [c_int, c_int, c_int, P, c_int, c_int, P, c_int, P, P, c_float, c_float, c_float, P,
                                P, c_int, c_int, P]),
    "tde_loss_l1": (c_int, [c_int, c_int, c_int, P, c_int, c_int, P, c_int, c_float, P, P, c_int, c_int, P]),
    "tde_adam_step_begin": (c_int, [P, P]),
    "tde_adam_update": (c_int, [c_size_t, P, P, P, P, P, c_float, c_float, c_float, c_float, c_float, P]),
    "tde_fill": (c_int, [c_size_t, P, c_float, P]),
    "tde_scale": (c_int, [c_size_t, P, c_float, P]),
    "tde_zero_bytes": (c_int, [c_size_t, P, P]),
    "tde_spatial_mean_fwd": (c_int, [c_int, c_int, c_int, P, c_int, P, P]),
    "tde_spatial_mean_bwd": (c_int, [c_int, c_int, c_int, P, c_int, c_int, P, P]),
    "tde_copy_view": (c_int, [c_int, c_int, P, c_int, c_int, P, c_int, c_int, c_int, P]),
}

_lib = None


class TdeError(RuntimeError):
    pass


def load(path=None):
    """Load libtde.so once; raise loudly if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("TDE_LIBRARY") or LIB_PATH   # override: A/B of kernel build variants
    if not os.path.exists(path):
        raise TdeError(f"libtde.so not built at {path}: run `make -C tf_depth_estimation_amd/csrc` "
                       "or __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.tde_abi_version()
    if v != ABI_VERSION:
        raise TdeError(f"libtde ABI {v} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS.keys())


def check(status, what=""):
    if status != 0:
        msg = _lib.tde_status_string(status).decode() if _lib is not None else str(status)
        raise TdeError(f"{what}: tde status {status} ({msg})")


def ptr(t):
    """Device pointer of a tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_hip = None
_own_streams = []


def dedicated_stream():
    """A HIP stream of its own (non-blocking) wrapped as a torch ExternalStream, kept for the life of the process.
    torch.cuda.Stream() hands out streams from a fixed round-robin pool, so after enough of them a "new" stream can
    be the very HIP stream a graph is being captured on or another side stream: a cross-stream wait between the two
    is then a self-wait.  (Stream priorities were measured in round 3 -- mixing priority classes cost up to 40 % --
    and are not offered.)"""
    s = ctypes.c_void_p()
    rc = hip().hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1))   # hipStreamNonBlocking
    if rc != 0 or not s.value:
        raise TdeError(f"hip stream creation failed ({rc})")
    _own_streams.append(s)
    return torch.cuda.ExternalStream(s.value)


def hip():
    """The HIP runtime (ctypes) for the few calls torch does not expose (dedicated streams)."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
    return _hip


# ---- cross-stream ordering inside stream capture
# torch's `a.wait_stream(b)` records a TEMPORARY event on b, waits on it and destroys it at once; inside a
# hipStreamBeginCapture region the capture's fork / join bookkeeping refers to that event.  The hot path's
# cross-stream waits go through wait_stream / wait_event below, which keep their events alive while any capture is
# open (capture_scope).  This was the first suspect for the config-4 single-graph capture_end segfault; it did not
# remove it: the bisection (probe/capture_bisect.py) pins that crash on a second-level fork (a stream
# forked from a captured stream that is not the capture origin), which the piece capture never makes.
_CAPTURE_DEPTH = [0]
_CAPTURE_EVENTS = []


_GC_WAS_ON = [False]


class capture_scope:
    """Context manager around every stream-capture region: events used for cross-stream waits inside it are kept,
    and Python's cyclic garbage collector is run once before the region and held off inside it.  A collection
    inside a capture can destroy an unreachable older trainer's graphs (hipGraphExecDestroy and the release of
    their memory pool, which frees device memory) while the capture is open: the process aborted that way in
    test_net_overlap_matches_serial (r03s2c, "Fatal Python error: Aborted" while "Garbage-collecting" under
    Trainer.capture).  torch.cuda.graph() collects before its own capture_begin but not inside; the piece and
    segmented captures call capture_begin directly."""

    def __enter__(self):
        if _CAPTURE_DEPTH[0] == 0:
            _GC_WAS_ON[0] = gc.isenabled()
            gc.collect()
            gc.disable()
            # graphs the collection destroyed (an older trainer's, possibly holding captured RCCL work whose
            # resources RCCL releases through graph user objects) are torn down with the device idle, before the
            # next capture begins
            if torch.cuda.is_initialized():
                torch.cuda.synchronize()
        _CAPTURE_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        _CAPTURE_DEPTH[0] -= 1
        if _CAPTURE_DEPTH[0] == 0:
            # every capture of the region has ended (its graph instantiated: a wait on an event recorded in the
            # same capture became a graph edge), so the kept events can go (they used to accumulate
            # for the life of the process, hundreds per capture)
            _CAPTURE_EVENTS.clear()
            if _GC_WAS_ON[0]:
                gc.enable()
        return False


def _keep(ev):
    if _CAPTURE_DEPTH[0] > 0:
        _CAPTURE_EVENTS.append(ev)


def wait_stream(waiter, waitee):
    """waiter waits for everything issued so far on waitee (torch's Stream.wait_stream, capture-safe)."""
    ev = torch.cuda.Event()
    ev.record(waitee)
    waiter.wait_event(ev)
    _keep(ev)


def wait_event(stream, ev):
    """stream waits on ev (capture-safe: ev kept alive while a capture is open)."""
    stream.wait_event(ev)
    _keep(ev)


def owned_stream(owner, name):
    """A dedicated stream (dedicated_stream) cached on `owner` under `name`: created once per owner and role, so
    re-enabling an overlap or re-capturing a step never allocates another HIP stream, and no two roles ever share
    one (the pool aliasing dedicated_stream avoids)."""
    cache = owner.__dict__.setdefault("_tde_streams", {})
    st = cache.get(name)
    if st is None:
        st = cache[name] = dedicated_stream()
    return st


def call(name, *args):
    """Call an int-returning ABI function and raise on a non-zero status."""
    lib = load()
    st = getattr(lib, name)(*args)
    check(st, name)
