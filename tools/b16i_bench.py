"""conv_halo_b16 (of_conv2d_b16i: bf16 image input, DMA-fed 16x32x128 tiles) against the
current bf16 kernels (of_conv2d_{fwd,dgrad}_bf16) on the decoder / encoder 3x3 shapes:
agreement (same bf16 operand rounding, fp32 summation order only) and time per launch.

python tools/b16i_bench.py [--batch 32] [--reps 20]   (GPU)
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from optical_flow_amd import _lib, ops  # noqa: E402
from optical_flow_amd._lib import ConvDesc, call  # noqa: E402

P = ops._ptr


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


def case(n, h, w, cin, cout, reps, lib):
    st = ops._stream()
    cin_p = (cin + 3) // 4 * 4
    cout_p = (cout + 3) // 4 * 4
    d = ConvDesc(n, h, w, cin, cin_p, cout, 3, 3, 1, 1, 1, h, w)
    wt = torch.randn(3, 3, cin, cout, device="cuda") * (2.0 / (9 * cin)) ** 0.5
    bias = torch.randn(cout, device="cuda") * 0.1
    wf = torch.empty(lib.of_conv_wfwd16_elems(C.byref(d)), dtype=torch.bfloat16, device="cuda")
    wb = torch.empty(lib.of_conv_wbwd16_elems(C.byref(d)), dtype=torch.bfloat16, device="cuda")
    call("of_conv_pack_weights_bf16", C.byref(d), P(wt), P(wf), P(wb), st)
    x = torch.zeros(n, h, w, cin_p, device="cuda")
    x[..., :cin] = torch.randn(n, h, w, cin, device="cuda")
    lx = (cin_p + 31) // 32 * 32
    x16 = torch.empty(n * h * w * lx, dtype=torch.bfloat16, device="cuda")
    call("of_to_bf16_image", P(x), n * h * w, cin_p, cin_p, P(x16), lx, st)
    y_ref = torch.empty(n, h, w, cout, device="cuda")
    y_new = torch.empty_like(y_ref)
    wsb = lib.of_conv2d_fwd_bf16_workspace(C.byref(d))
    ws = torch.empty(wsb // 4 + 4, device="cuda")
    ref_f = lambda: call("of_conv2d_fwd_bf16", C.byref(d), P(x), cin_p, P(wf), P(bias), None, None,
                         None, None, 0.0, None, cout, 2, 0.3, None, cout, P(y_ref), cout, P(ws),
                         wsb, st)
    new_f = lambda: call("of_conv2d_b16i", 0, C.byref(d), P(x16), lx, P(wf), P(bias), None, None,
                         None, None, 0.0, None, 0, None, 0, 2, 0.3, P(y_new), cout, st)
    ref_f()
    new_f()
    torch.cuda.synchronize()
    ef = ((y_new - y_ref).abs().max() / y_ref.abs().max()).item()
    tf_ref, tf_new = timeit(ref_f, reps), timeit(new_f, reps)
    flop = 2.0 * n * h * w * cin * cout * 9
    # dgrad
    dy = torch.zeros(n, h, w, cout_p, device="cuda")
    dy[..., :cout] = torch.randn(n, h, w, cout, device="cuda")
    ly = (cout_p + 31) // 32 * 32
    dy16 = torch.empty(n * h * w * ly, dtype=torch.bfloat16, device="cuda")
    call("of_to_bf16_image", P(dy), n * h * w, cout_p, cout_p, P(dy16), ly, st)
    src = torch.randn(n, h, w, cin_p, device="cuda")
    dx_ref = torch.empty(n, h, w, cin_p, device="cuda")
    dx_new = torch.empty_like(dx_ref)
    wsb2 = lib.of_conv2d_dgrad_bf16_workspace(C.byref(d))
    ws2 = torch.empty(wsb2 // 4 + 4, device="cuda")
    ref_d = lambda: call("of_conv2d_dgrad_bf16", C.byref(d), P(dy), cout_p, P(wb), P(src), cin_p,
                         2, 0.3, P(dx_ref), cin_p, P(ws2), wsb2, st)
    new_d = lambda: call("of_conv2d_b16i", 1, C.byref(d), P(dy16), ly, P(wb), None, None, None,
                         None, None, 0.0, None, 0, P(src), cin_p, 2, 0.3, P(dx_new), cin_p, st)
    ref_d()
    new_d()
    torch.cuda.synchronize()
    ed = ((dx_new - dx_ref).abs().max() / dx_ref.abs().max()).item()
    td_ref, td_new = timeit(ref_d, reps), timeit(new_d, reps)
    print("n%d %dx%d %d->%d | fwd err %.1e  ref %.3f ms (%.0f TF)  new %.3f ms (%.0f TF) | "
          "dgrad err %.1e  ref %.3f ms (%.0f TF)  new %.3f ms (%.0f TF)" % (
              n, h, w, cin, cout, ef, tf_ref, flop / tf_ref / 1e9, tf_new, flop / tf_new / 1e9,
              ed, td_ref, flop / td_ref / 1e9, td_new, flop / td_new / 1e9), flush=True)
    return ef, ed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    lib = _lib.load()
    n = args.batch
    worst = 0.0
    for (h, w, cin, cout) in [(192, 256, 128, 128), (192, 256, 115, 128), (96, 128, 128, 128),
                              (96, 128, 64, 64), (48, 64, 128, 128), (24, 32, 256, 256 // 2),
                              (37, 45, 20, 24)]:
        ef, ed = case(n, h, w, cin, cout, args.reps, lib)
        worst = max(worst, ef, ed)
    print("worst err %.2e" % worst)
    assert worst < 1e-4, worst


if __name__ == "__main__":
    main()
