"""Accuracy of the fp32 3x3 convs against an fp64 reference: the fp32 MFMA kernels
(of_conv2d_{fwd,dgrad}) and the split-bf16 kernels (of_conv2d_{fwd,dgrad}_x3) on the same
inputs.  Prints max |err| / max |ref| and rms(err) / rms(ref) per path.  GPU.

python tools/x3_accuracy.py
"""
import ctypes as C
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from optical_flow_amd import _lib, ops  # noqa: E402
from optical_flow_amd._lib import ACT_NONE, call  # noqa: E402

SHAPES = [(2, 48, 64, 128, 128), (2, 37, 45, 20, 24), (1, 96, 128, 64, 96), (2, 24, 32, 256, 256)]


def run(mode, n, h, w, cin, cout, x, wt, dy):
    layer = ops.ConvLayer(wt, torch.zeros(cout, device="cuda"), stride=1, act=ACT_NONE,
                          cin_p=cin, name="probe")
    d = layer.desc(n, h, w)
    layer._mode = mode
    wf, wd = layer.packed(d)
    P = ops._ptr
    st = ops._stream()
    y = torch.empty(n, h, w, cout, device="cuda")
    dx = torch.empty(n, h, w, cin, device="cuda")
    fent, fws = layer.fwd_entry(d)
    dent, dws = layer.dgrad_entry(d)
    fwt = torch.empty(fws // 4 + 4, device="cuda")
    dwt = torch.empty(dws // 4 + 4, device="cuda")
    call(fent, C.byref(d), P(x), cin, P(wf), P(layer.bias), None, None, None, None, 1e-3, None,
         0, ACT_NONE, 0.0, None, 0, P(y), cout, P(fwt), fws, st)
    call(dent, C.byref(d), P(dy), cout, P(wd), None, 0, ACT_NONE, 0.0, P(dx), cin, P(dwt), dws, st)
    torch.cuda.synchronize()
    return y.cpu().double(), dx.cpu().double()


def err(a, ref):
    e = a - ref
    return float(e.abs().max() / ref.abs().max()), float(e.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt())


def main():
    _lib.load()
    g = torch.Generator().manual_seed(0)
    for (n, h, w, cin, cout) in SHAPES:
        x = torch.randn(n, h, w, cin, generator=g)
        wt = torch.randn(3, 3, cin, cout, generator=g) * (2.0 / (9 * cin)) ** 0.5
        dy = torch.randn(n, h, w, cout, generator=g)
        xd, wdd, dyd = x.double(), wt.double(), dy.double()
        w_oihw = wdd.permute(3, 2, 0, 1)
        yref = F.conv2d(xd.permute(0, 3, 1, 2), w_oihw, padding=1).permute(0, 2, 3, 1)
        dxref = torch.nn.grad.conv2d_input((n, cin, h, w), w_oihw, dyd.permute(0, 3, 1, 2),
                                           padding=1).permute(0, 2, 3, 1)
        # fp32 CPU (sequential-ish fp32 arithmetic) for scale
        y32 = F.conv2d(x.permute(0, 3, 1, 2), wt.permute(3, 2, 0, 1), padding=1).permute(0, 2, 3, 1)
        line = "n%d %dx%d %d->%d | cpu-fp32 fwd %.2e/%.2e" % ((n, h, w, cin, cout) + err(y32.double(), yref))
        for mode, nm in ((0, "mfma-f32"), (2, "split-x3")):
            y, dx = run(mode, n, h, w, cin, cout, x.cuda(), wt.cuda(), dy.cuda())
            line += " | %s fwd %.2e/%.2e dgrad %.2e/%.2e" % ((nm,) + err(y, yref) + err(dx, dxref))
        print(line, flush=True)


if __name__ == "__main__":
    main()
