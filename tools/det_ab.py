"""Bitwise A/B of of_warp_bwd_det between two builds of liboflow.so (OFLOW_LIB): run once per
build with --out FILE, then --compare A B.  Shapes cover mode A (small flows, pile rows when
w - h > 16), mode B (smooth fields) and the fixed-point path, c = 16 / 64 / 128 / 96.

python tools/det_ab.py --out a.pt   (GPU);   python tools/det_ab.py --compare a.pt b.pt
"""
import argparse
import ctypes as C
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [  # (n, h, w, c, kind, scale, offset)
    (2, 48, 64, 64, "A", 2.0, 0.0), (1, 40, 90, 16, "A", 3.0, 0.0), (2, 64, 48, 128, "A", 1.5, 0.5),
    (1, 33, 47, 96, "A", 5.0, 0.0), (2, 48, 64, 64, "B", 3.0, 20.0), (1, 50, 70, 32, "B", 2.0, -15.0),
    (2, 48, 64, 64, "F", 30.0, 0.0), (8, 96, 128, 64, "A", 2.5, 0.0), (8, 192, 256, 64, "A", 2.0, 0.0),
]


def run(out):
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import call
    lib = _lib.lib()
    g = torch.Generator().manual_seed(5)
    res = []
    for n, h, w, c, kind, scale, off in CASES:
        f2 = torch.randn(n, h, w, c, generator=g).cuda()
        dg = torch.randn(n, h, w, c, generator=g).cuda()
        if kind == "B":
            ii, jj = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")
            fl = off + scale * torch.stack([torch.sin(0.21 * ii + 0.13 * jj),
                                            torch.cos(0.17 * ii - 0.11 * jj)], -1)
            fl = fl.expand(n, h, w, 2).contiguous().cuda()
        else:
            fl = (torch.randn(n, h, w, 2, generator=g) * scale + off).cuda()
        wsb = lib.of_warp_bwd_det_workspace(n, h, w, c)
        ws = torch.zeros((wsb + 3) // 4, dtype=torch.int32, device="cuda")
        dinp = torch.full((n, h, w, c), math.nan, device="cuda")
        dfl = torch.empty((n, h, w, 2), device="cuda")
        P = lambda t: C.c_void_p(t.data_ptr())
        call("of_warp_bwd_det", P(dg), P(f2), n, h, w, c, P(fl), 0, P(dinp), P(dfl), None, 0,
             P(ws), wsb, None)
        torch.cuda.synchronize()
        res.append((dinp.cpu(), dfl.cpu()))
    torch.save(res, out)


def compare(a, b):
    ra, rb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    ok = True
    for case, (x, y) in zip(CASES, zip(ra, rb)):
        same = torch.equal(x[0], y[0]) and torch.equal(x[1], y[1])
        ok &= same
        print(case, "bitwise equal" if same else "DIFFER max %.3g" % (x[0] - y[0]).abs().max())
    print("ALL EQUAL" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        sys.exit(compare(*args.compare))
    run(args.out)
