"""Microbenchmark of the conv kernels (fwd / dgrad / wgrad) on the flow net's layer shapes.

python tools/conv_bench.py [--reps 20]   (GPU)
Prints achieved TFLOP/s per (layer, pass) measured with torch.cuda events around `reps`
back-to-back launches on random data.
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from optical_flow_amd import _lib, ops  # noqa: E402
from optical_flow_amd._lib import ACT_LEAKY, ACT_NONE, ACT_RELU, call  # noqa: E402

# name, n, h, w, cin, cout, k, stride   (384x512, batch 8; encoder rows run on 2B = 16)
SHAPES = [
    ("dec3.c0", 8, 192, 256, 115, 128, 3, 1),
    ("dec3.c1", 8, 192, 256, 128, 128, 3, 1),
    ("dec3.c2", 8, 192, 256, 128, 96, 3, 1),
    ("dec3.c3", 8, 192, 256, 96, 64, 3, 1),
    ("dec3.c4", 8, 192, 256, 64, 32, 3, 1),
    ("dec3.c5", 8, 192, 256, 32, 2, 3, 1),
    ("dec2.c1", 8, 96, 128, 128, 128, 3, 1),
    ("dec1.c1", 8, 48, 64, 128, 128, 3, 1),
    ("enc.conv1", 16, 384, 512, 3, 64, 7, 2),
    ("enc.l2", 16, 96, 128, 64, 64, 3, 1),
    ("enc.l3.c0", 16, 96, 128, 64, 128, 3, 2),
    ("enc.l3.proj", 16, 96, 128, 64, 128, 1, 2),
    ("enc.l3", 16, 48, 64, 128, 128, 3, 1),
    ("enc.l4.c0", 16, 48, 64, 128, 256, 3, 2),
    ("enc.l4.proj", 16, 48, 64, 128, 256, 1, 2),
    ("enc.l4", 16, 24, 32, 256, 256, 3, 1),
]


def bench_one(name, n, h, w, cin, cout, k, s, reps, precision="fp32", cin_p=None):
    dev = "cuda"
    cin_p = cin_p or (cin + 3) // 4 * 4
    x = torch.randn(n, h, w, cin_p, device=dev)
    if cin_p != cin:
        x[..., cin:] = 0
    wt = torch.randn(k, k, cin, cout, device=dev) * (2.0 / (k * k * cin)) ** 0.5
    b = torch.randn(cout, device=dev) * 0.1
    layer = ops.ConvLayer(wt, b, stride=s, act=ACT_LEAKY, cin_p=cin_p, name=name,
                          precision=precision)
    d = layer.desc(n, h, w)
    wf, wd = layer.packed(d)
    cout_p = (cout + 3) // 4 * 4
    y = torch.empty(n, d.ho, d.wo, cout, device=dev)
    dy = torch.randn(n, d.ho, d.wo, cout_p, device=dev)
    dx = torch.empty_like(x)
    dw = torch.empty_like(wt)
    db = torch.empty_like(b)
    went, wsb = layer.wgrad_entry(d)
    ws = torch.empty(wsb // 4 + 1, device=dev)
    st = ops._stream()
    fent, fws = layer.fwd_entry(d)
    dent, dws = layer.dgrad_entry(d)
    fwt = torch.empty(fws // 4 + 4, device=dev)
    dwt = torch.empty(dws // 4 + 4, device=dev)
    P = ops._ptr
    flops = 2.0 * n * d.ho * d.wo * cout * k * k * cin

    def fwd():
        call(fent, C.byref(d), P(x), cin_p, P(wf), P(b), None, None, None, None,
             1e-3, None, 0, ACT_LEAKY, 0.3, None, 0, P(y), cout, P(fwt), fws, st)

    def dgrad():
        call(dent, C.byref(d), P(dy), cout_p, P(wd), P(x), cin_p, ACT_LEAKY, 0.3,
             P(dx), cin_p, P(dwt), dws, st)

    def wgrad():
        call(went, C.byref(d), P(x), cin_p, P(dy), cout_p, P(dw), P(db), 0, P(ws),
             wsb, st)

    out = {}
    for pname, fn in (("fwd", fwd), ("dgrad", dgrad), ("wgrad", wgrad)):
        if pname == "dgrad" and name == "enc.conv1":
            continue
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[pname] = (ms, flops / (ms * 1e-3) / 1e12)
    return flops, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--tune", default=None, help="key=value[,key=value] of_set_tuning")
    ap.add_argument("--bf16", action="store_true", help="bf16 MFMA fwd/dgrad/wgrad")
    ap.add_argument("--shapes", default=None,
                    help="extra shapes 'name:n,h,w,cin,cout,k,s[,cin_p];...' benched instead of SHAPES")
    args = ap.parse_args()
    shapes = SHAPES
    if args.shapes:
        shapes = []
        for item in args.shapes.split(";"):
            nm, dims = item.split(":")
            shapes.append((nm, *[int(v) for v in dims.split(",")]))
    _lib.load()
    if args.tune:
        for kv in args.tune.split(","):
            k, v = kv.split("=")
            _lib.lib().of_set_tuning(int(k), int(v))
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    # untimed pass over the first shape: the first timed layer otherwise reads 10-15 % slow
    # (clocks and caches still ramping; dec3.c0 116 vs the same shape benched again)
    bench_one(*shapes[0][:8], 3, "bf16" if args.bf16 else "fp32", *shapes[0][8:])
    for sh in shapes:
        if args.only and not any(o in sh[0] for o in args.only.split(",")):
            continue
        flops, out = bench_one(*sh[:8], args.reps, "bf16" if args.bf16 else "fp32",
                               *sh[8:])
        line = "%-10s %7.2f GF " % (sh[0], flops / 1e9)
        for p, (ms, tf) in out.items():
            line += " %s %7.3f ms %6.1f TF |" % (p, ms, tf)
            tot[p] += ms
        print(line, flush=True)
    print("total ms", {k: round(v, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
