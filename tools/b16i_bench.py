"""conv_halo_b16 (of_conv2d_b16i: bf16 activation images, DMA-fed 16x32-pixel tiles) against the
current bf16 kernels (of_conv2d_{fwd,dgrad}_bf16) on the decoder / encoder 3x3 shapes:
agreement (same bf16 operand rounding: fp32 summation order only) and time per launch, with
fp32 ends (the old kernels' interface) and with bf16-image ends (output image, act' from an
image, bias-gradient column sums).

python tools/b16i_bench.py [--batch 32] [--reps 20]   (GPU)
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from optical_flow_amd import _lib, ops  # noqa: E402
from optical_flow_amd._lib import B16iIO, ConvDesc, call  # noqa: E402

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


def img16(t, ld):
    n = t.numel() // t.shape[-1]
    out = torch.empty(n * ld, dtype=torch.bfloat16, device="cuda")
    call("of_to_bf16_image", P(t), n, t.shape[-1], t.shape[-1], P(out), ld, ops._stream())
    return out


def io(**kw):
    r = B16iIO()
    for k, v in kw.items():
        setattr(r, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
    return r


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


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
    flop = 2.0 * n * h * w * cin * cout * 9
    tf = lambda ms: flop / ms / 1e9
    # ---- forward
    x = torch.zeros(n, h, w, cin_p, device="cuda")
    x[..., :cin] = torch.randn(n, h, w, cin, device="cuda")
    lx = (cin_p + 31) // 32 * 32
    x16 = img16(x, lx)
    y_ref = torch.empty(n, h, w, cout, device="cuda")
    y_new = torch.empty_like(y_ref)
    y16 = torch.empty(n, h, w, cout, dtype=torch.bfloat16, device="cuda")
    wsb = lib.of_conv2d_fwd_bf16_workspace(C.byref(d))
    ws = torch.empty(wsb // 4 + 4, device="cuda")
    ref_f = lambda: call("of_conv2d_fwd_bf16", C.byref(d), P(x), cin_p, P(wf), P(bias), None, None,
                         None, None, 0.0, None, cout, 2, 0.3, None, cout, P(y_ref), cout, P(ws),
                         wsb, st)
    io32 = io(a16=x16, lda16=lx, y=y_new, ldy=cout)
    io16 = io(a16=x16, lda16=lx, y16=y16, ldy16=cout)
    new_f = lambda: call("of_conv2d_b16i", 0, C.byref(d), C.byref(io32), P(wf), P(bias), None,
                         None, None, None, 0.0, 2, 0.3, st)
    new_f16 = lambda: call("of_conv2d_b16i", 0, C.byref(d), C.byref(io16), P(wf), P(bias), None,
                           None, None, None, 0.0, 2, 0.3, st)
    ref_f()
    new_f()
    new_f16()
    torch.cuda.synchronize()
    assert torch.equal(y16, y_new.bfloat16()), "bf16 image != RNE of the fp32 output"
    ef = rel(y_new, y_ref)
    tf_ref, tf_new, tf_16 = timeit(ref_f, reps), timeit(new_f, reps), timeit(new_f16, reps)
    # ---- input gradient
    dy = torch.zeros(n, h, w, cout_p, device="cuda")
    dy[..., :cout] = torch.randn(n, h, w, cout, device="cuda")
    ly = (cout_p + 31) // 32 * 32
    dy16 = img16(dy, ly)
    src = torch.randn(n, h, w, cin_p, device="cuda")
    src16 = src.bfloat16()
    dx_ref = torch.empty(n, h, w, cin_p, device="cuda")
    dx_new = torch.empty_like(dx_ref)
    dx16 = torch.empty(n, h, w, cin_p, dtype=torch.bfloat16, device="cuda")
    tiles = lib.of_conv2d_b16i_tiles(1, C.byref(d))
    part = torch.empty(tiles, cin_p, device="cuda")
    db = torch.empty(cin_p, device="cuda")
    wsb2 = lib.of_conv2d_dgrad_bf16_workspace(C.byref(d))
    ws2 = torch.empty(wsb2 // 4 + 4, device="cuda")
    ref_d = lambda: call("of_conv2d_dgrad_bf16", C.byref(d), P(dy), cout_p, P(wb), P(src), cin_p,
                         2, 0.3, P(dx_ref), cin_p, P(ws2), wsb2, st)
    iod = io(a16=dy16, lda16=ly, y=dx_new, ldy=cin_p, act_src=src, ld_act=cin_p)
    iod16 = io(a16=dy16, lda16=ly, y16=dx16, ldy16=cin_p, act16=src16, ld_act16=cin_p,
               col_part=part)
    new_d = lambda: call("of_conv2d_b16i", 1, C.byref(d), C.byref(iod), P(wb), None, None, None,
                         None, None, 0.0, 2, 0.3, st)

    def new_d16():
        call("of_conv2d_b16i", 1, C.byref(d), C.byref(iod16), P(wb), None, None, None, None,
             None, 0.0, 2, 0.3, st)
        call("of_col_part_reduce", P(part), tiles, cin_p, P(db), 0, st)
    # direct epilogue: act' signs written by a forward producing this layer's input (mask_in)
    td_m = float("nan")
    if cin_p % 8 == 0 and cin_p == cin:
        dp = ConvDesc(n, h, w, 32, 32, cin, 3, 3, 1, 1, 1, h, w)
        wp = torch.randn(3, 3, 32, cin, device="cuda") * 0.1
        wfp = torch.empty(lib.of_conv_wfwd16_elems(C.byref(dp)), dtype=torch.bfloat16, device="cuda")
        wbp = torch.empty(lib.of_conv_wbwd16_elems(C.byref(dp)), dtype=torch.bfloat16, device="cuda")
        call("of_conv_pack_weights_bf16", C.byref(dp), P(wp), P(wfp), P(wbp), st)
        xp16 = torch.randn(n * h * w * 32, device="cuda").bfloat16()
        yp16 = torch.empty(n, h, w, cin, dtype=torch.bfloat16, device="cuda")
        mask = torch.empty(lib.of_conv2d_b16i_mask_bytes(C.byref(dp)) // 4, dtype=torch.int32,
                           device="cuda")
        call("of_conv2d_b16i", 0, C.byref(dp),
             C.byref(io(a16=xp16, lda16=32, y16=yp16, ldy16=cin, mask_out=mask)), P(wfp), None,
             None, None, None, None, 0.0, 2, 0.3, st)
        iodm = io(a16=dy16, lda16=ly, y16=dx16, ldy16=cin_p, mask_in=mask, col_part=part)

        def new_dm():
            call("of_conv2d_b16i", 1, C.byref(d), C.byref(iodm), P(wb), None, None, None, None,
                 None, 0.0, 2, 0.3, st)
            call("of_col_part_reduce", P(part), tiles, cin_p, P(db), 0, st)
        new_dm()
        td_m = timeit(new_dm, reps)
    ref_d()
    new_d()
    new_d16()
    torch.cuda.synchronize()
    assert torch.equal(dx16, dx_new.bfloat16()), "bf16 image != RNE of the fp32 output"
    ed = max(rel(dx_new, dx_ref), rel(db, dx_new.double().sum((0, 1, 2))))
    td_ref, td_new, td_16 = timeit(ref_d, reps), timeit(new_d, reps), timeit(new_d16, reps)
    # ---- weight gradient (x, dy as above)
    dw_ref = torch.empty(3, 3, cin, cout, device="cuda")
    db_ref = torch.empty(cout, device="cuda")
    dw_new = torch.empty_like(dw_ref)
    wsb3 = lib.of_conv2d_wgrad_bf16_workspace(C.byref(d))
    ws3 = torch.empty(wsb3 // 4 + 4, device="cuda")
    wsb4 = lib.of_conv2d_wgrad_b16i_workspace(C.byref(d))
    ws4 = torch.empty(wsb4 // 4 + 4, device="cuda")
    ref_w = lambda: call("of_conv2d_wgrad_bf16", C.byref(d), P(x), cin_p, P(dy), cout_p, P(dw_ref),
                         P(db_ref), 0, P(ws3), wsb3, st)
    new_w = lambda: call("of_conv2d_wgrad_b16i", C.byref(d), P(x16), lx, P(dy16), ly, P(dw_new), 0,
                         None, None, 0.0, P(ws4), wsb4, st)
    ref_w()
    new_w()
    torch.cuda.synchronize()
    ew = rel(dw_new, dw_ref)
    tw_ref, tw_new = timeit(ref_w, reps), timeit(new_w, reps)
    print("n%d %dx%d %d->%d | fwd err %.1e ref %.3f ms (%.0f TF) new %.3f (%.0f) bf16-out %.3f (%.0f)"
          " | dgrad err %.1e ref %.3f (%.0f) new %.3f (%.0f) bf16-ends+bias %.3f (%.0f)"
          " masks+bias %.3f (%.0f)"
          " | wgrad err %.1e ref %.3f (%.0f) new %.3f (%.0f)" % (
              n, h, w, cin, cout, ef, tf_ref, tf(tf_ref), tf_new, tf(tf_new), tf_16, tf(tf_16),
              ed, td_ref, tf(td_ref), td_new, tf(td_new), td_16, tf(td_16), td_m, tf(td_m),
              ew, tw_ref, tf(tw_ref), tw_new, tf(tw_new)), flush=True)
    if ABLATE:
        # timing ablations of conv_halo_b16 (of_set_tuning key 21; results are wrong): what the
        # epilogue's global traffic (1) and the main loop's DMAs (2) cost on this shape
        out = []
        for abl in (1, 2, 3):
            call("of_set_tuning", 21, abl)
            out.append((timeit(new_f16, reps), timeit(new_d16, reps)))
        call("of_set_tuning", 21, 0)
        print("   ablation (fwd16, dgrad16 ms): no-epilogue %.3f %.3f | no-DMA %.3f %.3f | neither"
              " %.3f %.3f" % tuple(v for p_ in out for v in p_), flush=True)
    return ef, max(ed, ew)


ABLATE = False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ablate", action="store_true")
    args = ap.parse_args()
    global ABLATE
    ABLATE = args.ablate
    lib = _lib.load()
    n = args.batch
    worst = 0.0
    for (h, w, cin, cout) in [(192, 256, 128, 128), (192, 256, 115, 128), (192, 256, 128, 96),
                              (192, 256, 96, 64), (192, 256, 64, 32), (96, 128, 128, 128),
                              (96, 128, 64, 64), (48, 64, 128, 128), (24, 32, 256, 256),
                              (37, 45, 20, 24)]:
        ef, ed = case(n, h, w, cin, cout, args.reps, lib)
        worst = max(worst, ef, ed)
    print("worst err %.2e" % worst)
    assert worst < 1e-4, worst


if __name__ == "__main__":
    main()
