"""Microbenchmark of the flow-specific kernels at the bench shapes (384x512, batch 8).

python tools/flow_bench.py [--reps 20]   (GPU)
Per flow-module level: cost-volume concat fwd / bwd and warp fwd / bwd, with the algorithmic
HBM bytes of each call and the achieved GB/s (torch.cuda events around `reps` launches).
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from optical_flow_amd import _lib, ops  # noqa: E402
from optical_flow_amd._lib import call  # noqa: E402

# level, h, w, c, cp (concat width), has_flow
LEVELS = [(3, 192, 256, 64, 116, True), (2, 96, 128, 64, 116, True),
          (1, 48, 64, 128, 180, True), (0, 24, 32, 256, 308, False)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--flow-scale", type=float, default=2.0,
                    help="std of the random flows in pixels (at init the net's are ~0.1)")
    ap.add_argument("--flow-offset", type=float, default=0.0,
                    help="constant added to both flow channels (large: clipped samples)")
    ap.add_argument("--corr-form", type=int, default=None,
                    help="of_set_tuning key 9 (cost-volume kernel forms; default: the library's)")
    args = ap.parse_args()
    _lib.load()
    if args.corr_form is not None:
        assert _lib.lib().of_set_tuning(9, args.corr_form) == 0
    n = args.batch
    P = ops._ptr
    st = ops._stream()
    tot = {}
    for lvl, h, w, c, cp, has_flow in LEVELS:
        f1 = torch.randn(n, h, w, c, device="cuda")
        f2 = torch.randn(n, h, w, c, device="cuda")
        fl = torch.randn(n, h, w, 2, device="cuda") * args.flow_scale + args.flow_offset if has_flow else None
        cat = torch.empty(n, h, w, cp, device="cuda")
        dcat = torch.randn(n, h, w, cp, device="cuda")
        df1, df2 = torch.empty_like(f1), torch.empty_like(f2)
        dfl = torch.empty(n, h, w, 2, device="cuda") if has_flow else None
        npx = n * h * w
        res = {}
        wsb = _lib.lib().of_corr_fwd_workspace(n, h, w, c, 3)
        ws = torch.empty(wsb // 4 + 4, device="cuda")
        res["corr_fwd"] = (timeit(lambda: call(
            "of_corr_concat_fwd", P(f1), P(f2), P(fl), n, h, w, c, 3, P(cat), cp, P(ws), wsb, st),
            args.reps),
            4 * npx * (2 * c + cp + (2 if has_flow else 0)))
        res["corr_bwd"] = (timeit(lambda: call(
            "of_corr_concat_bwd", P(dcat), cp, P(f1), P(f2), n, h, w, c, 3, P(df1), P(df2),
            P(dfl), st), args.reps), 4 * npx * (2 * (c + 49) + 4 * c + (4 if has_flow else 0)))
        if _lib.lib().of_set_tuning(9, 1) == 0:        # the two per-gradient kernels (r3)
            res["corr_bwd_sep"] = (timeit(lambda: call(
                "of_corr_concat_bwd", P(dcat), cp, P(f1), P(f2), n, h, w, c, 3, P(df1), P(df2),
                P(dfl), st), args.reps), res["corr_bwd"][1])
            _lib.lib().of_set_tuning(9, args.corr_form if args.corr_form is not None else 5)
        if has_flow:
            wout = torch.empty_like(f2)
            dw = torch.empty_like(f2)
            dfl2 = torch.empty(n, h, w, 2, device="cuda")
            res["warp_fwd"] = (timeit(lambda: call(
                "of_warp_fwd", P(f2), n, h, w, c, P(fl), P(wout), st), args.reps),
                4 * npx * (2 * c + 2))

            g = dcat[..., :c].contiguous()

            def wb2():
                call("of_fill", P(dw), 0.0, dw.numel(), st)
                call("of_warp_bwd", P(g), P(f2), n, h, w, c, P(fl), P(dw), P(dfl2), st)
            res["warp_bwd"] = (timeit(wb2, args.reps), 4 * npx * (4 * c + 4))
            dwsb = _lib.lib().of_warp_bwd_det_workspace(n, h, w, c)
            dws = torch.empty(dwsb // 4 + 4, device="cuda")
            res["warp_bwd_det"] = (timeit(lambda: call(
                "of_warp_bwd_det", P(g), P(f2), n, h, w, c, P(fl), 0, P(dw), P(dfl2), None, 0,
                P(dws), dwsb, st), args.reps), 4 * npx * (4 * c + 4))
        line = "level %d %3dx%3d c=%3d |" % (lvl, h, w, c)
        for k, (ms, by) in res.items():
            line += " %s %7.1f us %6.0f GB/s |" % (k, ms * 1e3, by / (ms * 1e-3) / 1e9)
            tot[k] = tot.get(k, 0.0) + ms
        print(line, flush=True)
    print("total us", {k: round(v * 1e3, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
