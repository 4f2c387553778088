"""Isolated timing of the BN backward reductions at the bench's B = 32, 384 x 512 sizes:
of_bn_bwd_reduce (layer1 size, with and without the t output) and the stem's fused
of_maxpool_bn_relu_bwd.  In the step these overlap the side stream's work, so their rocprof
durations include contention; this gives each one the whole chip.

    python tools/bn_bench.py [--reps 20]          (OFLOW_LIB=... for an A/B build)
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from optical_flow_amd._lib import call, lib  # noqa: E402

ACT_RELU = 1


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    P = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    dev = "cuda"
    c = 64
    vec = lambda: (1 + 0.1 * torch.rand(c, device=dev))
    gamma, beta, var = vec(), 0.1 * torch.randn(c, device=dev), vec()
    outs = [torch.zeros(c, device=dev) for _ in range(3)]

    for (h, w) in ((96, 128), (192, 256)):
        npix = 32 * h * w
        dy, y, res = (torch.randn(npix, c, device=dev) for _ in range(3))
        t = torch.empty(npix, c, device=dev)
        ws = torch.empty(lib().of_bn_act_bwd_workspace(npix, c) // 4 + 1, device=dev)
        for name, tout, nbytes in (("bn_bwd_reduce+t", t, 4), ("bn_bwd_reduce", None, 3)):
            us = timed(lambda: call("of_bn_bwd_reduce", npix, c, ACT_RELU, P(dy), P(y), P(res),
                                    P(gamma), P(beta), P(var), 1e-3, P(tout), P(outs[0]),
                                    P(outs[1]), P(outs[2]), 0, P(ws), None), a.reps)
            gb = nbytes * npix * c * 4 / 1e9
            print(f"{name:18s} {h}x{w} c={c} B=32  {us:8.1f} us  {gb / us * 1e6 / 1e3:6.2f} TB/s "
                  f"({gb:.3f} GB)")
        del dy, y, res, t, ws

    n, h, w = 32, 192, 256
    dyp = torch.randn(n, h // 2, w // 2, c, device=dev)
    g, y = torch.randn(n, h, w, c, device=dev), torch.randn(n, h, w, c, device=dev)
    dz = torch.empty(n, h, w, c, device=dev)
    ws = torch.empty(lib().of_maxpool_bn_act_bwd_workspace(n, h, w, c) // 4 + 1, device=dev)
    us = timed(lambda: call("of_maxpool_bn_relu_bwd", n, h, w, c, P(dyp), P(g), P(y), P(gamma),
                            P(beta), P(var), 1e-3, P(dz), P(outs[0]), P(outs[1]), P(outs[2]), 0,
                            P(ws), None), a.reps)
    gb = (3 * n * h * w * c + n * (h // 2) * (w // 2) * c) * 4 / 1e9
    print(f"{'maxpool_bn_relu':18s} {h}x{w} c={c} B=32  {us:8.1f} us  {gb / us * 1e6 / 1e3:6.2f} TB/s "
          f"({gb:.3f} GB)")


if __name__ == "__main__":
    main()
