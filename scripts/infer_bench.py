"""Inference-path measurement: batch_prediction.py's disp_net(is_training=False)
per-image latency at 224x224 batch 1, plus batched throughput, for the folded-BN graph predictor and the
unfolded (conv -> BN(moving) -> ReLU) path, graph and eager.  Prints one JSON line.

    python scripts/infer_bench.py [--iters 200] [--warmup 20]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tf_depth_estimation_amd import _api, _lib, batch_prediction, variables  # noqa: E402
from tf_depth_estimation_amd.program import conv_flops  # noqa: E402


def timed(pred, x, iters, warmup):
    for _ in range(warmup):
        pred(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        pred(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def flops(prog, N):
    from tf_depth_estimation_amd.program import ConvBN, Head
    return sum(conv_flops(op, N) for op in prog.spec.ops if isinstance(op, (ConvBN, Head)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--math", default="fp16x3", choices=list(_lib.CONV_MATH))
    args = ap.parse_args()
    lib = _lib.load()
    _lib.check(lib.tde_set_conv_math(_lib.CONV_MATH[args.math]))
    rows = []
    for net, H, W, B in [("disp_net", 224, 224, 1), ("disp_net", 192, 256, 8), ("disp_net", 192, 256, 64)]:
        for fold, graph in [(True, True), (False, True), (True, False)]:
            variables.get_store().reset(seed=1)
            _api.clear_programs()
            pred = batch_prediction.Predictor(net, H, W, batch=B, fold_bn=fold, graph=graph)
            x = torch.rand((B, H, W, 3), device="cuda") - 0.5
            iters = args.iters if B == 1 else max(20, args.iters // 4)
            s = timed(pred, x, iters, args.warmup)
            f = flops(pred.prog, B)
            rows.append({"net": net, "HxW": f"{H}x{W}", "batch": B, "fold_bn": fold, "hip_graph": graph,
                         "ms_per_call": round(s * 1e3, 4), "images_per_s": round(B / s, 1),
                         "conv_tflops": round(f / s / 1e12, 2)})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    # the whole loop body of batch_prediction.py:58-75 on the GPU: INTER_AREA of a decoded 480x640 uint8 image into
    # the 224x224 input, the folded-BN graph, INTER_CUBIC of disp1 to 240x720 and bilateralFilter(9, 75, 75); and
    # each OpenCV step alone (HIP events on the current stream)
    variables.get_store().reset(seed=1)
    _api.clear_programs()
    pred = batch_prediction.Predictor("disp_net", 224, 224, batch=1)
    img = torch.randint(0, 256, (1, 480, 640, 3), dtype=torch.uint8, device="cuda")
    s = timed(lambda x: pred.predict_depth_map(x, out_hw=(240, 720)), img, args.iters, args.warmup)
    post = {"chain_ms_per_image": round(s * 1e3, 4), "input": "480x640 uint8 -> 224x224 -> z 240x720"}
    d1 = pred.outs[0]
    z = batch_prediction.resize_cubic(d1, 240, 720)
    for name, fn, nbytes in (
            ("resize_area_u8 480x640x3 -> 224x224 (float view)",
             lambda: batch_prediction.resize_area(img, 224, 224, out_f32=pred.x), 480 * 640 * 3 + 224 * 224 * 12),
            ("resize_cubic 224x224 -> 240x720", lambda: batch_prediction.resize_cubic(d1, 240, 720, out=z),
             224 * 224 * 4 + 240 * 720 * 4),
            ("bilateral 240x720 d=9", lambda: batch_prediction.bilateral_filter(z, 9, 75.0, 75.0), 2 * 240 * 720 * 4)):
        for _ in range(args.warmup):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        post[name] = {"us": round(us, 2), "algorithmic_GBps": round(nbytes / (us * 1e-6) / 1e9, 1)}
    print(json.dumps(post), file=sys.stderr, flush=True)
    print(json.dumps({"metric": "disp_net inference (batch_prediction.py path)", "math": args.math,
                      "data": "synthetic U(-0.5,0.5) images, Glorot weights", "rows": rows,
                      "predict_depth_map": post}))


if __name__ == "__main__":
    main()
