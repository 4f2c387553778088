"""conv_tile_ws step timeline from s_memtime stamps (probe build: tools/ab_build.sh stamp
-DWS_STAMP with AB_SRCS=conv_ws.hip, run with OFLOW_LIB=.../ab_stamp/liboflow.so).

python tools/ws_probe.py [--mode fwd|dgrad] [--n 8 --h 192 --w 256 --cin 128 --cout 128]
Prints, for workgroup 0, per tap step: the compute waves' time from barrier to pre-barrier
(MFMA issue + own LDS reads), the barrier wait, and the B / halo waves' pre-barrier times.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from optical_flow_amd import _lib, ops  # noqa: E402
from optical_flow_amd._lib import ACT_LEAKY, call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fwd")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--h", type=int, default=192)
    ap.add_argument("--w", type=int, default=256)
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=128)
    args = ap.parse_args()
    lib = _lib.lib()
    assert lib.of_set_tuning(12, 2) == 0
    n, h, w, cin, cout = args.n, args.h, args.w, args.cin, args.cout
    x = torch.randn(n, h, w, cin, device="cuda")
    wt = torch.randn(3, 3, cin, cout, device="cuda") * 0.05
    b = torch.zeros(cout, device="cuda")
    dy = torch.randn(n, h, w, cout, device="cuda")
    layer = ops.ConvLayer(wt, b, act=ACT_LEAKY, cin_p=cin, precision="bf16")
    d = layer.desc(n, h, w)
    wf, wd = layer.packed(d)
    P, st = ops._ptr, ops._stream()
    y = torch.empty(n, h, w, cout, device="cuda")
    dx = torch.empty_like(x)
    fent, fws = layer.fwd_entry(d)
    dent, dws = layer.dgrad_entry(d)
    wsb = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
    for _ in range(3):
        if args.mode == "fwd":
            call(fent, C.byref(d), P(x), cin, P(wf), P(b), None, None, None, None, 1e-3, None, 0,
                 ACT_LEAKY, 0.3, None, 0, P(y), cout, P(wsb), fws, st)
        else:
            call(dent, C.byref(d), P(dy), cout, P(wd), P(x), cin, ACT_LEAKY, 0.3, P(dx), cin,
                 P(wsb), dws, st)
    torch.cuda.synchronize()
    buf = np.zeros(4 * 8 * 128, dtype=np.uint64)
    assert lib.of_ws_stamps(buf.ctypes.data_as(C.c_void_p)) == 0
    S = buf.reshape(4, 8, 128).astype(np.int64)
    for blk in range(2):
        T = S[blk]
        t0 = T[:, 0].min()
        steps = 0
        while steps < 41 and 3 * steps + 3 < 126 and T[0, 3 * steps + 3] != 0:
            steps += 1
        print("block %d: %d steps, loop end %d, epilogue %d cyc (wave 0)" % (
            blk, steps, T[0, 126] - t0, T[0, 127] - T[0, 126]))
        print("step  c.work  c.wait | B.issue B.vmwait B.wait | H.pre  H.store")
        for q in range(steps):
            cw = [T[wv, 3 * q + 2] - T[wv, 3 * q] for wv in range(4)]
            cwait = [T[wv, 3 * q + 3] - T[wv, 3 * q + 2] for wv in range(4)]
            bi = [T[wv, 3 * q + 1] - T[wv, 3 * q] for wv in (6, 7)]
            bv = [T[wv, 3 * q + 2] - T[wv, 3 * q + 1] for wv in (6, 7)]
            bw = [T[wv, 3 * q + 3] - T[wv, 3 * q + 2] for wv in (6, 7)]
            hp = [T[wv, 3 * q + 1] - T[wv, 3 * q] for wv in (4, 5)]
            hs = [T[wv, 3 * q + 2] - T[wv, 3 * q + 1] for wv in (4, 5)]
            print("%3d %6d %6d | %6d %6d %6d | %6d %6d   step %d" % (
                q, max(cw), max(cwait), max(bi), max(bv), max(bw), max(hp), max(hs),
                T[0, 3 * q + 3] - T[0, 3 * q]))


if __name__ == "__main__":
    main()
