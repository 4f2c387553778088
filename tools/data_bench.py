#!/usr/bin/env python
"""Throughput of the KITTI data path (SURVEY.md §8 f row 1) on synthetic KITTI-sized PNGs:

  decode     of_png_read_bgr, one host thread (frames/s)
  reader     AsyncReader.get_batch end to end (decode threads -> pinned slot -> H2D on a side
             stream -> of_preprocess_pairs), pairs/s, at --batch and --workers
  kernel     of_preprocess_pairs alone on a raw batch resident in HBM (hipEvents on its
             stream): us per launch and GB/s of algorithmic traffic (8-bit frames read once,
             float32 batch written once)

Frames: --frames synthetic 375x1242 BGR images (smooth gradients + texture + noise, so zlib
ratios are in the range of real street scenes), written with the native PNG encoder; pairs
cycle over them (the page cache holds the files, as it would for a hot dataset).
Prints one JSON line (and writes it to --out when given).
"""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synth_frame(rng, h, w):
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    base = np.stack([x / w * 180 + 40 * np.sin(y / 23.0), y / h * 200 + 30 * np.cos(x / 41.0),
                     (x + y) / (w + h) * 160 + 50], -1)
    tex = 25 * np.sin(x[..., None] / rng.uniform(3, 9) + y[..., None] / rng.uniform(4, 11))
    img = base + tex + rng.normal(0, 6, (h, w, 3))
    return np.clip(img, 0, 255).astype(np.uint8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from optical_flow_amd import _lib
    from optical_flow_amd._lib import call
    from optical_flow_amd.data_reader import AsyncReader, ReaderOpts, imread_bgr, imwrite
    _lib.load()
    rng = np.random.default_rng(0)
    tmp = tempfile.mkdtemp(prefix="ofdata_")
    paths = []
    png_bytes = 0
    for i in range(args.frames):
        p = os.path.join(tmp, "%010d.png" % i)
        imwrite(p, synth_frame(rng, 375, 1242))
        png_bytes += os.path.getsize(p)
        paths.append(p)
    res = {"frames": "%d synthetic 375x1242 PNGs, %.2f MB each" % (args.frames,
                                                                  png_bytes / args.frames / 1e6)}
    # ---- single-thread decode ----
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 2.0:
        imread_bgr(paths[n % len(paths)])
        n += 1
    res["decode_frames_per_s_1thread"] = round(n / (time.perf_counter() - t0), 1)

    # ---- AsyncReader end to end ----
    pairs = [[paths[i % len(paths)], paths[(i * 7 + 1) % len(paths)]] for i in range(args.pairs)]
    opts = ReaderOpts(None, args.batch, args.height, args.width, args.workers, seed=1, nslots=4,
                      pairs=pairs)
    with AsyncReader(opts) as r:
        for _ in range(3):
            r.get_batch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.batches):
            b = r.get_batch()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res["reader_pairs_per_s"] = round(args.batches * args.batch / dt, 1)
        res["reader_workers"] = args.workers
        raw_bytes = r.raw_bytes
    # ---- preprocess kernel alone, on a raw batch resident in HBM (host hand-out layout) ----
    with AsyncReader(ReaderOpts(None, args.batch, args.height, args.width, args.workers, seed=1,
                                nslots=1, pairs=pairs), pinned=False) as r2:
        raw = r2.next_raw()
    dev = torch.from_numpy(raw).cuda()
    out = torch.empty((args.batch, args.height, args.width, 6), device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(3):
        call("of_preprocess_pairs", C.c_void_p(dev.data_ptr()), args.batch, args.height,
             args.width, C.c_void_p(out.data_ptr()), C.c_void_p(s.cuda_stream))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record(s)
    for _ in range(reps):
        call("of_preprocess_pairs", C.c_void_p(dev.data_ptr()), args.batch, args.height,
             args.width, C.c_void_p(out.data_ptr()), C.c_void_p(s.cuda_stream))
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    alg = 2 * args.batch * 375 * 1242 * 3 + out.numel() * 4
    res["kernel_us"] = round(us, 2)
    res["kernel_alg_bytes"] = alg
    res["kernel_gbps"] = round(alg / (us * 1e-6) / 1e9, 1)
    res["kernel_frac_of_8tbps"] = round(alg / (us * 1e-6) / 8e12, 4)
    res["raw_batch_bytes"] = raw_bytes
    res["batch"] = args.batch
    res["out"] = [args.height, args.width]
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
