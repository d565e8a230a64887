"""Input-pipeline measurement: imageselect_Dataloader_optflow.DataLoader throughput on a
synthetic on-disk dataset, the resize/unpack kernel against the HBM roofline (HIP events on its stream), and a
config-2 training step fed by the loader (graph-replayed step + loader.load_train_batch + one device copy).

    python scripts/loader_bench.py [--batches 40] [--workers 16] [--shape ref|config2]

shape ref:     the reference loader's defaults: 240x1440 JPEG strips -> two 240x720 frames, 240x720 labels.
shape config2: the headline workload's frames: 192x512 strips -> two 192x256 frames, 192x256 labels.
Prints one JSON line."""
import argparse
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.dataset_util import make_dataset  # noqa: E402
from tf_depth_estimation_amd import _api, _lib, train, variables  # noqa: E402
from tf_depth_estimation_amd.imageselect_Dataloader_optflow import DataLoader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--shape", default="config2", choices=["ref", "config2"])
    ap.add_argument("--procs", type=int, default=16, help="JPEG decode worker processes (0: threads)")
    args = ap.parse_args()
    rh, rw = (240, 720) if args.shape == "ref" else (192, 256)
    B = args.batch
    tmp = tempfile.mkdtemp(prefix="tde_ds_")
    out = {"shape": args.shape, "frames": [rh, rw], "batch": B, "workers": args.workers, "decode_procs": args.procs}
    try:
        make_dataset(tmp, args.samples, strip_hw=(rh, 2 * rw), image_hw=(rh, rw), quality=90)
        # 1. loader alone: the consumer only waits for each batch to be resident
        dl = DataLoader(tmp, B, rh, rw, 2, 4, "train", resizedheight=rh, resizedwidth=rw, seed=0,
                        workers=args.workers, prefetch=3, decode_procs=args.procs)
        for _ in range(5):
            dl.load_train_batch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.batches):
            dl.load_train_batch()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out["loader_samples_per_s"] = round(B * args.batches / dt, 1)

        # 2. the device kernel alone, timed with HIP events on its stream (the loader's last slot re-run)
        slot = dl._held
        a = _lib.ImageBatch()
        a.B, a.out_h, a.out_w, a.nframes = B, rh, rw, 2
        base = slot.dev.data_ptr()
        a.src, a.src_off, a.src_hw = base, base, base + 8 * B
        a.out[0], a.out[1] = slot.tgt.data_ptr(), slot.src.data_ptr()
        a.out_cstride[0] = a.out_cstride[1] = 3
        lib = _lib.load()
        n = 50
        g = torch.cuda.CUDAGraph()     # n launches captured: the HIP events then time the kernel, not the host
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            lib.tde_image_resize_unpack(ctypes.byref(a), _lib.stream_ptr())
        torch.cuda.current_stream().wait_stream(cs)
        with torch.cuda.graph(g):
            for _ in range(n):
                lib.tde_image_resize_unpack(ctypes.byref(a), _lib.stream_ptr())
        g.replay()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        # algorithmic bytes per launch: the decoded strips read once + both float frames written
        nbytes = B * (rh * 2 * rw * 3) + 2 * B * rh * rw * 3 * 4
        out["kernel_us"] = round(us, 2)
        out["kernel_bytes"] = nbytes
        out["kernel_GBps"] = round(nbytes / us / 1e3, 1)
        out["kernel_frac_hbm"] = round(nbytes / us / 1e3 / 8000.0, 4)
        dl.close()

        # 3. config-2 training fed by the loader (only at the headline frame size)
        if args.shape == "config2":
            variables.get_store().reset(seed=1)
            _api.clear_programs()
            tr = train.DepthOnlyTrainer(B, rh, rw)
            tr.enable_wgrad_overlap()
            dl = DataLoader(tmp, B, rh, rw, 2, 4, "train", resizedheight=rh, resizedwidth=rw, seed=1,
                            workers=args.workers, prefetch=3, decode_procs=args.procs)
            tgt, src, label, *_ = dl.load_train_batch()
            tr.set_batch(tgt, label)
            tr.capture(warmup=2)

            def run(k, feed):
                for _ in range(k):
                    if feed:
                        tgt, src, label, *_ = dl.load_train_batch()
                        tr.images.copy_(tgt)
                        tr.label.copy_(label)
                    tr.step()
            run(10, True)
            torch.cuda.synchronize()
            for feed, key in ((False, "train_synthetic"), (True, "train_fed")):
                t0 = time.perf_counter()
                run(args.batches, feed)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                out[key] = round(B * args.batches / dt, 1)
            # the same with a 0.2 ms GIL switch interval (the consumer thread launches each step sooner while
            # the loader's threads hold the GIL; a process-wide setting, so only measured here)
            sw = sys.getswitchinterval()
            sys.setswitchinterval(2e-4)
            t0 = time.perf_counter()
            run(args.batches, True)
            torch.cuda.synchronize()
            out["train_fed_switch_0.2ms"] = round(B * args.batches / (time.perf_counter() - t0), 1)
            sys.setswitchinterval(sw)
            dl.close()
        out["host_cpus"] = os.cpu_count()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
