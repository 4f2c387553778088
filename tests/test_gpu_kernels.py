"""Per-kernel parity: every HIP kernel through the C ABI vs the CPU oracle (float64) on the
same seeded inputs.  Tolerance: 1e-3 relative (REL_TOL), per BASELINE.json's north star."""
import zlib
import pytest
import torch

from helpers import REL_TOL, dev, f64, rel_inf, rel_l2, rng_tensor
from oracle import ref_flow as R

pytestmark = pytest.mark.gpu


def _ops():
    from optical_flow_amd import ops
    return ops


# ------------------------------------------------------------------------------- conv ----
CONV_CASES = [
    # (n, h, w, cin, cout, k, stride, act, bn, residual)
    (2, 16, 24, 16, 32, 3, 1, "leaky", False, False),
    (2, 16, 24, 115, 128, 3, 1, "leaky", False, False),     # decoder c0 (cin padded)
    (1, 12, 16, 32, 2, 3, 1, "none", False, False),         # flow conv (cout 2): narrow path
    (2, 33, 70, 32, 2, 3, 1, "none", False, False),         # narrow, ragged, many slices
    (3, 40, 100, 32, 4, 3, 1, "leaky", False, False),       # narrow tiled, cout 4, ragged
    (1, 9, 33, 32, 1, 3, 1, "relu", False, False),          # narrow tiled, cout 1
    (8, 96, 512, 32, 2, 3, 1, "leaky", False, False),       # narrow tiled: 2 tiles per wgrad block
    (6, 128, 320, 32, 4, 3, 1, "none", False, False),       # narrow tiled: 1-2 tiles per block
    (2, 17, 65, 32, 3, 3, 1, "none", False, False),         # narrow tiled, cout 3
    (1, 10, 20, 64, 3, 3, 1, "relu", False, False),         # narrow, 16 lanes per pixel
    (2, 8, 8, 3, 2, 3, 1, "leaky", False, False),           # narrow, 1 lane per pixel
    (1, 9, 9, 12, 2, 3, 1, "leaky", False, False),          # cin_p 12: GEMM fallback
    (2, 20, 36, 64, 64, 3, 1, "relu", True, True),          # wgrad tiles <2,2> (fp32 too)
    # smoke() level 1 (64x128 image, batch 1): 32-pixel layers, deep split-K
    (1, 4, 8, 179, 128, 3, 1, "leaky", False, False),
    (1, 4, 8, 128, 96, 3, 1, "leaky", False, False),
    (1, 4, 8, 32, 2, 3, 1, "none", False, False),
    (2, 16, 16, 64, 96, 3, 1, "leaky", False, False),       # cout 96 tile
    (2, 32, 48, 3, 64, 7, 2, "relu", True, False),          # conv1 7x7/2 + BN + ReLU
    (2, 16, 16, 64, 128, 3, 2, "relu", True, False),        # stride-2 block conv
    (2, 16, 16, 64, 128, 1, 2, "none", True, False),        # 1x1/2 projection + BN
    (2, 8, 8, 128, 128, 3, 1, "relu", True, True),          # conv_b + BN + residual + ReLU
    (1, 6, 10, 256, 256, 3, 1, "relu", True, False),        # odd sizes, 2 n-tiles
    (3, 9, 7, 20, 40, 3, 2, "leaky", False, False),         # odd spatial, stride 2
]


@pytest.mark.parametrize("split", [True, False], ids=["x3", "f32"])
@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: "x".join(map(str, c[:7])) + c[7])
def test_conv_fwd_bwd(case, split):
    """split: 3x3 stride-1 fwd/dgrad on the split-bf16 kernels (the fp32 default) or on the
    fp32 MFMA implicit GEMM; other shapes take the same kernels either way."""
    ops = _ops()
    from optical_flow_amd._lib import ACT_LEAKY, ACT_NONE, ACT_RELU
    n, h, w, cin, cout, k, s, act, use_bn, use_res = case
    seed = zlib.crc32(repr(case).encode()) % 1000   # (hash() of str is salted per process)
    if act != "none":
        # Reseed until no pre-activation sits within 1e-4 of the ReLU/LeakyReLU kink, where a
        # 1-ulp fp32 difference would flip the derivative (a data property, not a kernel bug).
        for _ in range(20):
            xx = rng_tensor((n, h, w, cin), seed)
            ww = rng_tensor((k, k, cin, cout), seed + 1, scale=(2.0 / (k * k * cin)) ** 0.5)
            pre = R.conv2d_same(f64(xx), f64(ww), f64(rng_tensor((cout,), seed + 2, scale=0.1)), s)
            if use_bn:
                pre = R.batchnorm_inference(pre, {
                    "bn/gamma": f64(rng_tensor((cout,), seed + 3, lo=0.5, hi=1.5)),
                    "bn/beta": f64(rng_tensor((cout,), seed + 4, scale=0.1)),
                    "bn/moving_mean": f64(rng_tensor((cout,), seed + 5, scale=0.1)),
                    "bn/moving_variance": f64(rng_tensor((cout,), seed + 6, lo=0.5, hi=1.5))}, "bn")
            if use_res:
                pre = pre + f64(rng_tensor(tuple(pre.shape), seed + 7))
            if pre.abs().min().item() > 1e-4:
                break
            seed += 1000
    x = rng_tensor((n, h, w, cin), seed)
    wt = rng_tensor((k, k, cin, cout), seed + 1, scale=(2.0 / (k * k * cin)) ** 0.5)
    b = rng_tensor((cout,), seed + 2, scale=0.1)
    g = rng_tensor((cout,), seed + 3, lo=0.5, hi=1.5)
    be = rng_tensor((cout,), seed + 4, scale=0.1)
    mu = rng_tensor((cout,), seed + 5, scale=0.1)
    var = rng_tensor((cout,), seed + 6, lo=0.5, hi=1.5)
    # --- oracle
    xo, wo_, bo, go, beo = [f64(t).requires_grad_(True) for t in (x, wt, b, g, be)]
    zo = R.conv2d_same(xo, wo_, bo, s)
    yo = zo
    p = {"bn/gamma": go, "bn/beta": beo, "bn/moving_mean": f64(mu), "bn/moving_variance": f64(var)}
    if use_bn:
        yo = R.batchnorm_inference(yo, p, "bn")
    res = rng_tensor(tuple(yo.shape), seed + 7) if use_res else None
    reso = f64(res).requires_grad_(True) if use_res else None
    if use_res:
        yo = yo + reso
    yo = {"relu": torch.relu, "leaky": R.leaky_relu, "none": lambda t: t}[act](yo)
    gy = rng_tensor(tuple(yo.shape), seed + 8)
    (yo * f64(gy)).sum().backward()
    # --- device
    cin_p = (cin + 3) // 4 * 4
    xd = torch.zeros((n, h, w, cin_p), device="cuda")
    xd[..., :cin] = dev(x)
    wd, bd, gd, bed = [dev(t).requires_grad_(True) for t in (wt, b, g, be)]
    layer = ops.ConvLayer(wd, bd, stride=s,
                          act={"relu": ACT_RELU, "leaky": ACT_LEAKY, "none": ACT_NONE}[act],
                          bn=(gd, bed, dev(mu), dev(var)) if use_bn else None, cin_p=cin_p,
                          f32_split=split)
    if split and k == 3 and s == 1 and cout > 4:
        assert layer.mode(layer.desc(n, h, w)) == 2
    xd.requires_grad_(True)
    resd = dev(res).requires_grad_(True) if use_res else None
    yd = layer(xd, residual=resd)
    assert yd.shape == yo.shape
    assert rel_inf(yd, yo) < REL_TOL, "forward"
    (yd * dev(gy)).sum().backward()
    torch.cuda.synchronize()
    assert rel_inf(xd.grad[..., :cin], xo.grad) < REL_TOL, "dgrad"
    if cin < cin_p:
        assert xd.grad[..., cin:].abs().max().item() == 0.0, "padded channels must get 0 grad"
    assert rel_l2(wd.grad, wo_.grad) < REL_TOL, "wgrad"
    assert rel_l2(bd.grad, bo.grad) < REL_TOL, "bias grad"
    if use_bn:
        assert rel_l2(gd.grad, go.grad) < REL_TOL, "gamma grad"
        assert rel_l2(bed.grad, beo.grad) < REL_TOL, "beta grad"
    if use_res:
        assert rel_inf(resd.grad, reso.grad) < REL_TOL, "residual grad"


BF16_CASES = [c for c in CONV_CASES if c[4] > 4] + [
    (8, 64, 128, 128, 128, 3, 1, "leaky", False, False),  # halo tiles, large grid
    (2, 48, 64, 256, 256, 3, 1, "relu", True, True),      # K split, BN + residual
    (1, 13, 35, 48, 64, 3, 1, "leaky", False, False),    # halo tiles: ragged, partial chunk
    (1, 8, 16, 256, 128, 3, 1, "relu", True, False),     # halo tiles: split over channels
    (2, 40, 70, 64, 64, 3, 1, "leaky", False, False),    # wgrad tiles <2,2>: ragged, splits
    (1, 24, 48, 128, 96, 3, 1, "leaky", False, False),   # wgrad tiles <1,4>: partial co tile
    (1, 17, 20, 64, 32, 3, 1, "leaky", False, False),    # wgrad tiles <2,2>: cout 32
]


@pytest.mark.parametrize("case", BF16_CASES, ids=lambda c: "x".join(map(str, c[:7])) + c[7])
def test_conv_bf16(case):
    """bf16 MFMA fwd/dgrad (configs 3-5) against the float64 oracle on bf16-rounded operands."""
    ops = _ops()
    from optical_flow_amd._lib import ACT_LEAKY, ACT_NONE, ACT_RELU
    n, h, w, cin, cout, k, s, act, use_bn, use_res = case
    seed = zlib.crc32(repr(case).encode()) % 1000 + 17   # stable across processes
    x = rng_tensor((n, h, w, cin), seed)
    wt = rng_tensor((k, k, cin, cout), seed + 1, scale=(2.0 / (k * k * cin)) ** 0.5)
    b = rng_tensor((cout,), seed + 2, scale=0.1)
    g = rng_tensor((cout,), seed + 3, lo=0.5, hi=1.5)
    be = rng_tensor((cout,), seed + 4, scale=0.1)
    mu = rng_tensor((cout,), seed + 5, scale=0.1)
    var = rng_tensor((cout,), seed + 6, lo=0.5, hi=1.5)
    xo, wo_, bo = [f64(t).requires_grad_(True) for t in (x, wt, b)]
    if use_bn:     # the folded-BN rounding points of the build (oracle _Bf16ConvBN)
        yo = R._Bf16ConvBN.apply(xo, wo_, bo, f64(g), f64(be), f64(mu), f64(var), s)
    else:
        yo = R._Bf16Conv.apply(xo, wo_, bo, s)
    res = rng_tensor(tuple(yo.shape), seed + 7) if use_res else None
    if use_res:
        yo = yo + f64(res)
    yo = {"relu": torch.relu, "leaky": R.leaky_relu, "none": lambda t: t}[act](yo)
    gy = rng_tensor(tuple(yo.shape), seed + 8)
    (yo * f64(gy)).sum().backward()
    cin_p = (cin + 3) // 4 * 4
    xd = torch.zeros((n, h, w, cin_p), device="cuda")
    xd[..., :cin] = dev(x)
    wd, bd = [dev(t).requires_grad_(True) for t in (wt, b)]
    layer = ops.ConvLayer(wd, bd, stride=s,
                          act={"relu": ACT_RELU, "leaky": ACT_LEAKY, "none": ACT_NONE}[act],
                          bn=(dev(g), dev(be), dev(mu), dev(var)) if use_bn else None,
                          cin_p=cin_p, precision="bf16")
    assert layer.bf16()
    xd.requires_grad_(True)
    yd = layer(xd, residual=dev(res) if use_res else None)
    assert rel_inf(yd, yo) < REL_TOL, "forward"
    (yd * dev(gy)).sum().backward()
    torch.cuda.synchronize()
    assert rel_inf(xd.grad[..., :cin], xo.grad) < REL_TOL, "dgrad"
    if cin < cin_p:
        assert xd.grad[..., cin:].abs().max().item() == 0.0, "padded channels must get 0 grad"
    assert rel_l2(wd.grad, wo_.grad) < REL_TOL, "wgrad"
    assert rel_l2(bd.grad, bo.grad) < REL_TOL, "bias grad"


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 48, 64, 128, 128), (2, 37, 45, 20, 24),
                                             (1, 96, 128, 64, 96), (2, 24, 32, 256, 256)])
def test_conv_x3_accuracy(n, h, w, cin, cout):
    """The split-bf16 fp32 kernels are as accurate as the fp32 MFMA kernels: error against
    an fp64 reference (max and rms, relative to the reference) within 3x of theirs and at
    the level of one fp32 rounding per product (tools/x3_accuracy.py prints the numbers)."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd._lib import ACT_NONE, call
    x = rng_tensor((n, h, w, cin), 11)
    wt = rng_tensor((3, 3, cin, cout), 12, scale=(2.0 / (9 * cin)) ** 0.5)
    dy = rng_tensor((n, h, w, cout), 13)
    yref = R.conv2d_same(f64(x), f64(wt), None, 1)
    dxref = torch.nn.grad.conv2d_input((n, cin, h, w), f64(wt).permute(3, 2, 0, 1),
                                       f64(dy).permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    errs = {}
    for split in (False, True):
        layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=1, act=ACT_NONE, cin_p=cin,
                              f32_split=split)
        d = layer.desc(n, h, w)
        assert layer.mode(d) == (2 if split else 0)
        wf, wd = layer.packed(d)
        fent, fws = layer.fwd_entry(d)
        dent, dws = layer.dgrad_entry(d)
        ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
        P, st = ops._ptr, ops._stream()
        xd, dyd = dev(x), dev(dy)
        y = torch.empty(n, h, w, cout, device="cuda")
        dx = torch.empty(n, h, w, cin, device="cuda")
        call(fent, C.byref(d), P(xd), cin, P(wf), P(layer.bias), None, None, None, None, 1e-3,
             None, 0, ACT_NONE, 0.0, None, 0, P(y), cout, P(ws), fws, st)
        call(dent, C.byref(d), P(dyd), cout, P(wd), None, 0, ACT_NONE, 0.0, P(dx), cin, P(ws),
             dws, st)
        torch.cuda.synchronize()
        errs[split] = [rel_inf(y, yref), rel_l2(y, yref), rel_inf(dx, dxref), rel_l2(dx, dxref)]
    for e3, e32 in zip(errs[True], errs[False]):
        assert e3 < 3 * e32 + 1e-7, (errs[True], errs[False])
        assert e3 < 5e-6, errs[True]


@pytest.mark.parametrize("n,h,w,cin,cout,k,s", [(4, 64, 96, 4, 64, 7, 2),   # stem (cin 3 -> 4)
                                               (4, 48, 64, 64, 128, 3, 2),   # res3_0 conv_a
                                               (4, 24, 32, 128, 256, 3, 2),  # res4_0 conv_a
                                               (4, 48, 64, 64, 128, 1, 2)])  # projection
def test_conv_gemm_x3_accuracy(n, h, w, cin, cout, k, s, monkeypatch):
    """The split-bf16 implicit GEMMs (conv_gemm_x3 fwd / dgrad with phase groups,
    conv_wgrad_x3: stem, stride-2 and 1x1 layers) are as accurate as the fp32 MFMA kernels:
    against fp64, within 3x of the fp32 MFMA kernel's error and at the level of one fp32
    rounding per product."""
    import ctypes as C
    ops = _ops()
    monkeypatch.setattr(ops, "X3_GEMM_MIN_CIN", 0)   # the stem shape too (the model keeps it fp32)
    from optical_flow_amd._lib import ACT_NONE, call
    x = rng_tensor((n, h, w, cin), 91)
    wt = rng_tensor((k, k, cin, cout), 92, scale=(2.0 / (k * k * cin)) ** 0.5)
    errs = {}
    for split in (False, True):
        layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=s, act=ACT_NONE, cin_p=cin,
                              f32_split=split)
        d = layer.desc(n, h, w)
        assert layer.mode(d) == (2 if split else 0)
        dy = rng_tensor((n, d.ho, d.wo, cout), 93)
        pad = (d.pad_top, d.pad_left)
        yref = R.conv2d_same(f64(x), f64(wt), None, s)
        wf, wd = layer.packed(d)
        fent, fws = layer.fwd_entry(d)
        dent, dws = layer.dgrad_entry(d)
        ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
        P, st = ops._ptr, ops._stream()
        xd, dyd = dev(x), dev(dy)
        y = torch.empty(n, d.ho, d.wo, cout, device="cuda")
        dx = torch.empty(n, h, w, cin, device="cuda")
        call(fent, C.byref(d), P(xd), cin, P(wf), P(layer.bias), None, None, None, None, 1e-3,
             None, 0, ACT_NONE, 0.0, None, 0, P(y), cout, P(ws), fws, st)
        e = [rel_inf(y, yref), rel_l2(y, yref)]
        went, wws = layer.wgrad_entry(d)
        wsw = torch.empty(wws // 4 + 4, device="cuda")
        dw = torch.empty(k, k, cin, cout, device="cuda")
        call(went, C.byref(d), P(xd), cin, P(dyd), cout, P(dw), None, 0, P(wsw), wws, st)
        wo = f64(wt).requires_grad_(True)
        (R.conv2d_same(f64(x), wo, None, s) * f64(dy)).sum().backward()
        e += [rel_inf(dw, wo.grad), rel_l2(dw, wo.grad)]
        if k < 7:
            call(dent, C.byref(d), P(dyd), cout, P(wd), None, 0, ACT_NONE, 0.0, P(dx), cin, P(ws),
                 dws, st)
            xo = f64(x).requires_grad_(True)
            (R.conv2d_same(xo, f64(wt), None, s) * f64(dy)).sum().backward()
            e += [rel_inf(dx, xo.grad), rel_l2(dx, xo.grad)]
        torch.cuda.synchronize()
        errs[split] = e
        assert pad is not None
    for e3, e32 in zip(errs[True], errs[False]):
        assert e3 < 3 * e32 + 1e-7, (errs[True], errs[False])
        assert e3 < 5e-6, errs[True]


@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("n,h,w,cin,cout,k,s", [(4, 48, 64, 64, 128, 3, 2),   # res3_0 conv_a
                                               (4, 24, 32, 128, 256, 3, 2),  # res4_0 conv_a
                                               (4, 48, 64, 64, 128, 1, 2),   # projection
                                               (3, 37, 45, 20, 40, 3, 2),    # odd, 64-col tiles
                                               (1, 6, 10, 8, 16, 3, 2),      # 1-3 chunks
                                               (2, 64, 96, 4, 64, 7, 2)])    # stem shape
def test_conv_gemm_x3_ring_bitwise(n, h, w, cin, cout, k, s, prec, monkeypatch):
    """conv_gemm_x3 on the LDS-DMA rings (of_set_tuning key 30 = 1: 3 slots, one chunk in flight
    across each barrier; key 30 = 2, the default: 2 slots, two workgroups per CU; A and B by
    DMA, A split / rounded as it is read) equals the register-staged form (key 30 = 0) bit for bit -- forward and the stride-2 input gradient's
    phase groups, split-K and unsplit grids, rings of 1-3 chunks -- for the fp32 split (three
    planes) and the bf16 (one plane) kernels; the timing kinds say the GEMMs ran."""
    import ctypes as C
    if k == 7 and prec == "bf16":
        pytest.skip("the bf16 stem shape runs conv_gemm_bf16 (conv_gemm_x3<..., 1> takes no stem)")
    ops = _ops()
    monkeypatch.setattr(ops, "X3_GEMM_MIN_CIN", 0)
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_NONE, call
    lib = _lib.lib()
    x = rng_tensor((n, h, w, cin), 111)
    wt = rng_tensor((k, k, cin, cout), 112, scale=(2.0 / (k * k * cin)) ** 0.5)
    kw = dict(precision="bf16") if prec == "bf16" else dict(f32_split=True)
    layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=s, act=ACT_NONE, cin_p=cin,
                          **kw)
    d = layer.desc(n, h, w)
    dy = rng_tensor((n, d.ho, d.wo, cout), 113)
    wf, wd = layer.packed(d)
    P, st = ops._ptr, ops._stream()
    xd, dyd = dev(x), dev(dy)
    res = {}
    try:
        assert lib.of_set_tuning(8, 0) == 0           # the fp32 stem shape on the GEMM
        assert lib.of_set_tuning(16, 7) == 0          # bf16 forward on conv_gemm_x3<..., 1> too
        for ring in (1, 2, 0):
            assert lib.of_set_tuning(30, ring) == 0
            fent, fws = layer.fwd_entry(d)
            dent, dws = layer.dgrad_entry(d)
            ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
            y = torch.full((n, d.ho, d.wo, cout), float("nan"), device="cuda")
            dx = torch.full((n, h, w, cin), float("nan"), device="cuda")
            lib.of_timing_enable(1)
            call(fent, C.byref(d), P(xd), cin, P(wf), P(layer.bias), None, None, None, None,
                 1e-3, None, 0, ACT_NONE, 0.0, None, 0, P(y), cout, P(ws), fws, st)
            if k < 7:
                call(dent, C.byref(d), P(dyd), cout, P(wd), None, 0, ACT_NONE, 0.0, P(dx), cin,
                     P(ws), dws, st)
            torch.cuda.synchronize()
            kk = (C.c_int * 64)()
            cnt = lib.of_timing_read(64, kk, None, None)
            lib.of_timing_enable(0)
            res[ring] = (y, dx, {kk[i] for i in range(cnt)})
    finally:
        lib.of_set_tuning(30, 2)
        lib.of_set_tuning(16, 6)
        lib.of_set_tuning(8, 1)
        lib.of_timing_enable(0)
    base = 240 if prec == "bf16" else 160
    want = {base + (0 if cout > 64 else 1)}
    if k < 7:
        want.add(base + 8 + (0 if cin > 64 else 1))
    for ring in (1, 2):
        assert want <= res[ring][2] and want <= res[0][2], (want, res[ring][2], res[0][2])
        assert torch.isfinite(res[ring][0]).all()
        assert torch.equal(res[ring][0], res[0][0])
        if k < 7:
            assert torch.isfinite(res[ring][1]).all()
            assert torch.equal(res[ring][1], res[0][1])


@pytest.mark.parametrize("n,h,w", [(2, 64, 96), (1, 50, 70), (2, 38, 130)])
def test_conv_stem_x3(n, h, w):
    """The stem forward on its own split-bf16 kernel (conv_stem_x3: 7x7 stride 2, 3 -> 4
    input channels, 64 outputs; bias, BN, ReLU and z in the epilogue; ragged output tiles)
    against fp64 and against conv_gemm_x3 (of_set_tuning key 8 = 0), as accurate as one fp32
    rounding per product; the 32- and 64-channel workgroup forms (key 8 = 1, 2) bitwise equal;
    the timing kind says which kernel ran."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_RELU, call
    lib = _lib.lib()
    cin, cout = 4, 64
    xc = rng_tensor((n, h, w, 3), 61)
    x = torch.cat([xc, torch.zeros(n, h, w, 1)], -1)
    wt = rng_tensor((7, 7, 3, cout), 62, scale=(2.0 / 147) ** 0.5)
    wp = torch.cat([wt, torch.zeros(7, 7, 1, cout)], 2)
    b = rng_tensor((cout,), 63, scale=0.1)
    g, be = rng_tensor((cout,), 64, scale=0.5) + 1.0, rng_tensor((cout,), 65, scale=0.1)
    mu, var = rng_tensor((cout,), 66, scale=0.1), rng_tensor((cout,), 67).abs() + 0.5
    layer = ops.ConvLayer(dev(wt), dev(b), stride=2, act=ACT_RELU, cin_p=cin, f32_split=True)
    d = layer.desc(n, h, w)
    assert layer.mode(d) == 2
    wf, _ = layer.packed(d)
    fent, fws = layer.fwd_entry(d)
    ws = torch.empty(fws // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    xd, bd, gd, bed, mud, vard = [dev(t) for t in (x, b, g, be, mu, var)]
    outs, kinds = [], []
    try:
        for form in (1, 2, 0):
            assert lib.of_set_tuning(8, form) == 0
            y = torch.full((n, d.ho, d.wo, cout), 7.0, device="cuda")
            z = torch.full((n, d.ho, d.wo, cout), 7.0, device="cuda")
            lib.of_timing_enable(1)
            call(fent, C.byref(d), P(xd), cin, P(wf), P(bd), P(gd), P(bed), P(mud), P(vard), 1e-3,
                 None, 0, ACT_RELU, 0.0, P(z), cout, P(y), cout, P(ws), fws, st)
            torch.cuda.synchronize()
            lib.of_timing_enable(0)
            kk = (C.c_int * 16)()
            fl = (C.c_double * 16)()
            ms = (C.c_float * 16)()
            cnt = lib.of_timing_read(16, kk, fl, ms)
            kinds.append({kk[i] for i in range(cnt)})
            outs.append((y, z))
    finally:
        lib.of_set_tuning(8, 1)
        lib.of_timing_enable(0)
    assert kinds[0] == {184} and kinds[1] == {184} and 184 not in kinds[2], kinds
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    zref = R.conv2d_same(f64(x), f64(wp), f64(b), 2)
    yref = torch.relu((zref - f64(mu)) / torch.sqrt(f64(var) + 1e-3) * f64(g) + f64(be))
    for (y, z) in outs:
        assert rel_inf(z, zref) < 5e-6 and rel_inf(y, yref) < 5e-6, (rel_inf(z, zref), rel_inf(y, yref))
    assert rel_l2(outs[0][0], yref) < 3 * rel_l2(outs[2][0], yref) + 1e-7


@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("n,h,w", [(2, 64, 96), (1, 50, 70), (8, 384, 512)])
def test_conv_stem_persistent_bitwise(n, h, w, prec):
    """conv_stem_x3 persistent over tiles (of_set_tuning key 31: the default workgroups per CU,
    and 1) against one tile per workgroup (key 31 = 0): y, z and the max-pooled output
    (of_conv2d_fwd_pool) bit for bit, fp32 (three planes) and bf16 (one plane), ragged tiles
    and the bench size (12 tiles per workgroup)."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_RELU, call
    lib = _lib.lib()
    cin, cout = 4, 64
    xc = rng_tensor((n, h, w, 3), 71)
    x = torch.cat([xc, torch.zeros(n, h, w, 1)], -1)
    wt = rng_tensor((7, 7, 3, cout), 72, scale=(2.0 / 147) ** 0.5)
    b = rng_tensor((cout,), 73, scale=0.1)
    g, be = rng_tensor((cout,), 74, scale=0.5) + 1.0, rng_tensor((cout,), 75, scale=0.1)
    mu, var = rng_tensor((cout,), 76, scale=0.1), rng_tensor((cout,), 77).abs() + 0.5
    kw = dict(precision="bf16") if prec == "bf16" else dict(f32_split=True)
    layer = ops.ConvLayer(dev(wt), dev(b), stride=2, act=ACT_RELU, cin_p=cin, **kw)
    d = layer.desc(n, h, w)
    m = layer.mode(d)
    wf, _ = layer.packed(d)
    fent, fws = layer.fwd_entry(d)
    ws = torch.empty(fws // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    xd, bd, gd, bed, mud, vard = [dev(t) for t in (x, b, g, be, mu, var)]
    outs = []
    try:
        for per_cu in (0, -1, 1):
            assert lib.of_set_tuning(31, per_cu) == 0
            y = torch.full((n, d.ho, d.wo, cout), 7.0, device="cuda")
            z = torch.full((n, d.ho, d.wo, cout), 7.0, device="cuda")
            call(fent, C.byref(d), P(xd), cin, P(wf), P(bd), P(gd), P(bed), P(mud), P(vard), 1e-3,
                 None, 0, ACT_RELU, 0.0, P(z), cout, P(y), cout, P(ws), fws, st)
            yp = torch.full((n, d.ho, d.wo, cout), 7.0, device="cuda")
            xp = torch.full((n, d.ho // 2, d.wo // 2, cout), 7.0, device="cuda")
            pooled = d.ho % 2 == 0 and d.wo % 2 == 0
            if pooled:
                _lib.check(lib.of_conv2d_fwd_pool(
                    C.byref(d), m, P(xd), cin, P(wf), P(bd), P(gd), P(bed), P(mud), P(vard),
                    C.c_float(1e-3), ACT_RELU, C.c_float(0.0), None, cout, P(yp), cout, P(xp),
                    P(ws), fws, st), "of_conv2d_fwd_pool")
            torch.cuda.synchronize()
            outs.append((y, z, yp, xp, pooled))
    finally:
        lib.of_set_tuning(31, -1)
    y0, z0, yp0, xp0, pooled = outs[0]
    assert torch.isfinite(y0).all() and (y0 != 7.0).any()
    for y, z, yp, xp, _ in outs[1:]:
        assert torch.equal(y, y0) and torch.equal(z, z0)
        if pooled:
            assert torch.equal(yp, yp0) and torch.equal(xp, xp0) and torch.equal(yp0, y0)


@pytest.mark.parametrize("n,h,w,cin,cout,k,s", [(4, 48, 64, 64, 128, 3, 2),    # res3_0 conv_a
                                               (4, 24, 32, 128, 256, 3, 2),   # res4_0 conv_a
                                               (4, 48, 64, 64, 128, 1, 2),    # projection
                                               (3, 37, 45, 20, 40, 3, 2),     # odd, 64-col tiles
                                               (2, 64, 96, 4, 64, 7, 2),      # stem, key 15 = 0
                                               (64, 96, 128, 64, 128, 3, 2)])  # bench B = 32 size
def test_conv_gemm_b16_forms(n, h, w, cin, cout, k, s):
    """The bf16 implicit GEMMs on the one-plane split-kernel forms (conv_gemm_x3<..., 1> fwd /
    dgrad with phase groups, conv_wgrad_x3<..., 1>; of_set_tuning key 16 = 1) against
    conv_gemm_bf16 / conv_wgrad_bf16 (key 16 = 0): the same bf16-rounded products, fp32 sums
    in another order; both within the bf16 tolerance of the float64 oracle on bf16-rounded
    operands; the timing kinds say which kernels ran."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_NONE, call
    lib = _lib.lib()
    x = rng_tensor((n, h, w, cin), 101)
    wt = rng_tensor((k, k, cin, cout), 102, scale=(2.0 / (k * k * cin)) ** 0.5)
    layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=s, act=ACT_NONE, cin_p=cin,
                          precision="bf16")
    d = layer.desc(n, h, w)
    dy = rng_tensor((n, d.ho, d.wo, cout), 103)
    wf, wd = layer.packed(d)
    P, st = ops._ptr, ops._stream()
    xd, dyd = dev(x), dev(dy)

    def kinds():
        kk = (C.c_int * 64)()
        cnt = lib.of_timing_read(64, kk, None, None)
        return {kk[i] for i in range(cnt)}

    res = {}
    try:
        assert lib.of_set_tuning(15, 0) == 0          # the stem shape on the GEMMs as well
        for form in (1, 0):
            assert lib.of_set_tuning(16, 7 if form else 0) == 0
            fent, fws = layer.fwd_entry(d)
            dent, dws = layer.dgrad_entry(d)
            went, wws = layer.wgrad_entry(d)
            ws = torch.empty(max(fws, dws, wws) // 4 + 4, device="cuda")
            y = torch.empty(n, d.ho, d.wo, cout, device="cuda")
            dx = torch.empty(n, h, w, cin, device="cuda")
            dw = torch.empty(k, k, cin, cout, device="cuda")
            lib.of_timing_enable(1)
            call(fent, C.byref(d), P(xd), cin, P(wf), P(layer.bias), None, None, None, None,
                 1e-3, None, 0, ACT_NONE, 0.0, None, 0, P(y), cout, P(ws), fws, st)
            if k < 7:
                call(dent, C.byref(d), P(dyd), cout, P(wd), None, 0, ACT_NONE, 0.0, P(dx), cin,
                     P(ws), dws, st)
            call(went, C.byref(d), P(xd), cin, P(dyd), cout, P(dw), None, 0, P(ws), wws, st)
            torch.cuda.synchronize()
            res[form] = (y, dx if k < 7 else None, dw, kinds())
            lib.of_timing_enable(0)
    finally:
        lib.of_set_tuning(16, 6)
        lib.of_set_tuning(15, 1)
        lib.of_timing_enable(0)
    want = {240 + (0 if cout > 64 else 1), 256 + (0 if cout > 64 else 1)}
    if k < 7:                                        # (the input gradient's N is cin)
        want.add(248 + (0 if cin > 64 else 1))
    assert want <= res[1][3] and not {kk for kk in res[0][3] if kk >= 240}, (res[1][3], res[0][3])
    # the two kernel families differ only in fp32 summation order
    assert rel_inf(res[1][0], res[0][0]) < 1e-5
    assert rel_l2(res[1][2], res[0][2]) < 1e-5
    if k < 7:
        assert rel_inf(res[1][1], res[0][1]) < 1e-5
    if n * h * w > 300000:
        return      # (the bench size: A/B agreement only, no float64 oracle on the host)
    xo = f64(x).requires_grad_(True)
    wo = f64(wt).requires_grad_(True)
    yref = R._Bf16Conv.apply(xo, wo, None, s)
    (yref * f64(dy)).sum().backward()
    for form in (1, 0):
        y, dx, dw = res[form][:3]
        assert rel_inf(y, yref) < REL_TOL, (form, rel_inf(y, yref))
        assert rel_l2(dw, wo.grad) < REL_TOL, (form, rel_l2(dw, wo.grad))
        if dx is not None:
            assert rel_inf(dx, xo.grad) < REL_TOL, (form, rel_inf(dx, xo.grad))


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 40, 70, 64, 64), (1, 24, 48, 128, 96),
                                             (8, 96, 128, 128, 128), (2, 17, 20, 64, 32),
                                             (4, 64, 96, 115, 128), (8, 128, 256, 128, 128)])
def test_conv_bf16_prefetch_forms(n, h, w, cin, cout):
    """The bf16 3x3 kernels with their MFMA fragments read ahead (conv_tile_bf16 PF = 1,
    of_set_tuning key 20; conv_wgrad_tile_bf16 PF = 1, key 17; the defaults) do the same MFMAs
    in the same order as the round-1 schedules (keys = 0): forward, input and weight gradients
    bitwise equal, on every channel-tile form, ragged tiles and the tall forward tiles."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, call
    lib = _lib.lib()
    cin_p = (cin + 3) // 4 * 4
    x = torch.zeros(n, h, w, cin_p)
    x[..., :cin] = rng_tensor((n, h, w, cin), 121)
    wt = rng_tensor((3, 3, cin, cout), 122, scale=(2.0 / (9 * cin)) ** 0.5)
    layer = ops.ConvLayer(dev(wt), dev(rng_tensor((cout,), 123, scale=0.1)), stride=1,
                          act=ACT_LEAKY, cin_p=cin_p, precision="bf16")
    d = layer.desc(n, h, w)
    cout_p = (cout + 3) // 4 * 4
    dy = torch.zeros(n, h, w, cout_p)
    dy[..., :cout] = rng_tensor((n, h, w, cout), 124)
    xd, dyd = dev(x), dev(dy)
    wf, wd = layer.packed(d)
    P, st = ops._ptr, ops._stream()
    res = {}
    try:
        for form in (1, 0):
            assert lib.of_set_tuning(17, form) == 0 and lib.of_set_tuning(20, form) == 0
            fent, fws = layer.fwd_entry(d)
            dent, dws = layer.dgrad_entry(d)
            went, wws = layer.wgrad_entry(d)
            ws = torch.empty(max(fws, dws, wws) // 4 + 4, device="cuda")
            y = torch.empty(n, h, w, cout, device="cuda")
            dx = torch.empty(n, h, w, cin_p, device="cuda")
            dw = torch.empty(3, 3, cin, cout, device="cuda")
            db = torch.empty(cout, device="cuda")
            call(fent, C.byref(d), P(xd), cin_p, P(wf), P(layer.bias), None, None, None, None,
                 1e-3, None, 0, ACT_LEAKY, 0.3, None, 0, P(y), cout, P(ws), fws, st)
            call(dent, C.byref(d), P(dyd), cout_p, P(wd), P(xd), cin_p, ACT_LEAKY, 0.3, P(dx),
                 cin_p, P(ws), dws, st)
            call(went, C.byref(d), P(xd), cin_p, P(dyd), cout_p, P(dw), P(db), 0, P(ws), wws, st)
            torch.cuda.synchronize()
            res[form] = [t.cpu() for t in (y, dx, dw, db)]
    finally:
        lib.of_set_tuning(17, 1)
        lib.of_set_tuning(20, 1)
    for a_, b_, what in zip(res[1], res[0], ("fwd", "dgrad", "wgrad", "bias grad")):
        assert torch.equal(a_, b_), what


# Every conv_halo_b16 N tile (128 / 96 / 64 / 32) and conv_wgrad_b16i form (Cout tile 128 /
# 64 / 32: (2,4) / (4,2) / (4,1) waves), ragged tiles and padded channels.
B16I_CASES = [(2, 40, 70, 128, 128), (1, 37, 45, 20, 24), (2, 24, 48, 128, 96),
              (2, 32, 40, 96, 64), (2, 20, 36, 64, 32), (1, 16, 32, 256, 256), (3, 17, 33, 115, 128)]


@pytest.mark.parametrize("n,h,w,cin,cout", B16I_CASES)
def test_conv_b16i(n, h, w, cin, cout, b16i_persist):
    """The bf16-activation-image 3x3 kernels (of_conv2d_b16i fwd / dgrad, of_conv2d_wgrad_b16i)
    through the C ABI against float64 convolutions of the same bf16-rounded operands (the
    oracle's bf16 rounding points, R._Bf16Conv): forward with bias + LeakyReLU, input gradient
    with the producer's act' from an fp32 or a bf16 source and the bias-gradient column sums,
    weight gradient; fp32 and bf16-image outputs (the image is the RNE of the fp32 output)."""
    import ctypes as C
    import torch.nn.functional as Fn
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, B16iIO, ConvDesc, call
    lib = _lib.load()
    P, st = ops._ptr, ops._stream()
    seed = zlib.crc32(repr((n, h, w, cin, cout)).encode()) % 1000
    cin_p, cout_p = (cin + 3) // 4 * 4, (cout + 3) // 4 * 4
    lx, ly = (cin_p + 31) // 32 * 32, (cout_p + 31) // 32 * 32
    d = ConvDesc(n, h, w, cin, cin_p, cout, 3, 3, 1, 1, 1, h, w)
    bf = lambda t: f64(t.to(torch.bfloat16).float())
    nchw = lambda t: t.permute(0, 3, 1, 2)
    nhwc = lambda t: t.permute(0, 2, 3, 1)

    def img16(t, c, ld):
        out = torch.zeros(t.numel() // t.shape[-1] * ld, dtype=torch.bfloat16, device="cuda")
        call("of_to_bf16_image", P(t), t.numel() // t.shape[-1], c, t.shape[-1], P(out), ld, st)
        return out

    def io(**kw):
        r = B16iIO()
        for k, v in kw.items():
            setattr(r, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
        return r

    x = rng_tensor((n, h, w, cin), seed)
    wt = rng_tensor((3, 3, cin, cout), seed + 1, scale=(2.0 / (9 * cin)) ** 0.5)
    bias = rng_tensor((cout,), seed + 2, scale=0.1)
    dy = rng_tensor((n, h, w, cout), seed + 3)
    src = rng_tensor((n, h, w, cin), seed + 4)
    wk = bf(wt).permute(3, 2, 0, 1).contiguous()                  # (cout, cin, 3, 3)
    y_o = nhwc(Fn.conv2d(nchw(bf(x)), wk, f64(bias), padding=1))
    y_o = torch.where(y_o > 0, y_o, 0.3 * y_o)
    slope = torch.where(f64(src) > 0, 1.0, 0.3).double()
    dx_o = nhwc(torch.nn.grad.conv2d_input((n, cin, h, w), wk, nchw(bf(dy)), padding=1)) * slope
    dw_o = torch.nn.grad.conv2d_weight(nchw(bf(x)), wk.shape, nchw(bf(dy)), padding=1)
    dw_o = dw_o.permute(2, 3, 1, 0)                                # (3, 3, cin, cout)

    wd = dev(wt)
    wf = torch.empty(lib.of_conv_wfwd16_elems(C.byref(d)), dtype=torch.bfloat16, device="cuda")
    wb = torch.empty(lib.of_conv_wbwd16_elems(C.byref(d)), dtype=torch.bfloat16, device="cuda")
    call("of_conv_pack_weights_bf16", C.byref(d), P(wd), P(wf), P(wb), st)
    xd = torch.zeros(n, h, w, cin_p, device="cuda")
    xd[..., :cin] = dev(x)
    dyd = torch.zeros(n, h, w, cout_p, device="cuda")
    dyd[..., :cout] = dev(dy)
    srcd = torch.zeros(n, h, w, cin_p, device="cuda")
    srcd[..., :cin] = dev(src)
    x16, dy16 = img16(xd, cin_p, lx), img16(dyd, cout_p, ly)
    bd = dev(bias)
    # forward: fp32 output and bf16 image
    y32 = torch.empty(n, h, w, cout, device="cuda")
    y16 = torch.empty(n, h, w, cout, dtype=torch.bfloat16, device="cuda")
    for o in (io(a16=x16, lda16=lx, y=y32, ldy=cout), io(a16=x16, lda16=lx, y16=y16, ldy16=cout)):
        call("of_conv2d_b16i", 0, C.byref(d), C.byref(o), P(wf), P(bd), None, None, None, None,
             0.0, ACT_LEAKY, 0.3, st)
    # input gradient: act' from the fp32 source / from its bf16 image with the column sums
    dx32 = torch.empty(n, h, w, cin_p, device="cuda")
    dx16 = torch.empty(n, h, w, cin_p, dtype=torch.bfloat16, device="cuda")
    src16 = srcd.bfloat16()
    tiles = lib.of_conv2d_b16i_tiles(1, C.byref(d))
    part = torch.empty(tiles, cin_p, device="cuda")
    db = torch.empty(cin_p, device="cuda")
    call("of_conv2d_b16i", 1, C.byref(d),
         C.byref(io(a16=dy16, lda16=ly, y=dx32, ldy=cin_p, act_src=srcd, ld_act=cin_p)), P(wb),
         None, None, None, None, None, 0.0, ACT_LEAKY, 0.3, st)
    call("of_conv2d_b16i", 1, C.byref(d),
         C.byref(io(a16=dy16, lda16=ly, y16=dx16, ldy16=cin_p, act16=src16, ld_act16=cin_p,
                    col_part=part)), P(wb), None, None, None, None, None, 0.0, ACT_LEAKY, 0.3, st)
    call("of_col_part_reduce", P(part), tiles, cin_p, P(db), 0, st)
    # no activation (the first head conv's input gradient): the direct fp32 epilogue
    dxn = torch.empty(n, h, w, cin_p, device="cuda")
    call("of_conv2d_b16i", 1, C.byref(d), C.byref(io(a16=dy16, lda16=ly, y=dxn, ldy=cin_p)),
         P(wb), None, None, None, None, None, 0.0, 0, 0.0, st)
    # weight gradient
    dw = torch.empty(3, 3, cin, cout, device="cuda")
    wsb = lib.of_conv2d_wgrad_b16i_workspace(C.byref(d))
    ws = torch.empty(wsb // 4 + 4, device="cuda")
    call("of_conv2d_wgrad_b16i", C.byref(d), P(x16), lx, P(dy16), ly, P(dw), 0, None, None, 0.0,
         P(ws), wsb, st)
    torch.cuda.synchronize()
    tol = 1e-4                     # same bf16 operands: fp32 summation order only
    assert rel_inf(y32, y_o) < tol, "forward"
    assert torch.equal(y16, y32.bfloat16()), "forward image != RNE of the fp32 output"
    assert rel_inf(dx32[..., :cin], dx_o) < tol, "dgrad"
    assert dx32[..., cin:].abs().max().item() == 0.0 if cin < cin_p else True
    assert torch.equal(dx16, dx32.bfloat16()), "dgrad image != RNE of the fp32 output"
    assert rel_l2(db[:cin], f64(dx32[..., :cin]).sum((0, 1, 2))) < tol, "column sums"
    assert rel_inf(dxn[..., :cin], dx_o / slope) < tol, "dgrad, no activation"
    assert rel_l2(dw, dw_o) < tol, "wgrad"


@pytest.fixture(params=[0, 2], ids=["tile", "persist"])
def b16i_persist(request):
    """conv_halo_b16 one tile per workgroup, or persistent on 8 workgroups (of_set_tuning key 24
    = 2: multi-tile walks at test sizes, the next tile's loads in flight during the epilogue)."""
    from optical_flow_amd import _lib
    lib = _lib.lib()
    assert lib.of_set_tuning(24, request.param) == 0
    yield request.param
    lib.of_set_tuning(24, 0)


@pytest.mark.parametrize("n,h,w,c0,c1,c2", [(2, 40, 70, 115, 128, 128), (1, 37, 45, 64, 96, 64),
                                             (2, 20, 36, 96, 64, 32), (1, 16, 32, 128, 32, 64),
                                             (4, 48, 96, 64, 128, 96)])
def test_conv_b16i_direct_masks(n, h, w, c0, c1, c2, b16i_persist):
    """conv_halo_b16's direct epilogue (bf16 image output alone): layer A (c0 -> c1) forward
    writes its output image and its act' signs (mask_out); the input gradient of layer B
    (c1 -> c2) reads the signs (mask_in).  Against the general epilogue (of_set_tuning key 22
    = 0 for the forward; act_src = A's fp32 output for the gradient): the images bitwise, the
    bias-gradient column sums to fp32 summation order."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, B16iIO, ConvDesc, call
    lib = _lib.load()
    P, st = ops._ptr, ops._stream()
    seed = zlib.crc32(repr((n, h, w, c0, c1, c2)).encode()) % 1000
    l0, l1, l2 = [(c + 31) // 32 * 32 for c in ((c0 + 3) // 4 * 4, c1, c2)]
    dA = ConvDesc(n, h, w, c0, (c0 + 3) // 4 * 4, c1, 3, 3, 1, 1, 1, h, w)
    dB = ConvDesc(n, h, w, c1, c1, c2, 3, 3, 1, 1, 1, h, w)

    def io(**kw):
        r = B16iIO()
        for k, v in kw.items():
            setattr(r, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
        return r

    def packed(d, cin, cout, sd):
        wt = dev(rng_tensor((3, 3, cin, cout), sd, scale=(2.0 / (9 * cin)) ** 0.5))
        wf = torch.empty(lib.of_conv_wfwd16_elems(C.byref(d)), dtype=torch.bfloat16, device="cuda")
        wb = torch.empty(lib.of_conv_wbwd16_elems(C.byref(d)), dtype=torch.bfloat16, device="cuda")
        call("of_conv_pack_weights_bf16", C.byref(d), P(wt), P(wf), P(wb), st)
        return wf, wb

    wfA, _ = packed(dA, c0, c1, seed + 1)
    _, wbB = packed(dB, c1, c2, seed + 2)
    bias = dev(rng_tensor((c1,), seed + 3, scale=0.1))
    x = torch.zeros(n, h, w, (c0 + 3) // 4 * 4, device="cuda")
    x[..., :c0] = dev(rng_tensor((n, h, w, c0), seed))
    x16 = torch.zeros(n * h * w * l0, dtype=torch.bfloat16, device="cuda")
    call("of_to_bf16_image", P(x), n * h * w, x.shape[-1], x.shape[-1], P(x16), l0, st)
    dy = torch.zeros(n, h, w, c2, device="cuda")
    dy[...] = dev(rng_tensor((n, h, w, c2), seed + 4))
    dy16 = torch.zeros(n * h * w * l2, dtype=torch.bfloat16, device="cuda")
    call("of_to_bf16_image", P(dy), n * h * w, c2, c2, P(dy16), l2, st)
    mask = torch.empty(lib.of_conv2d_b16i_mask_bytes(C.byref(dA)) // 4, dtype=torch.int32,
                       device="cuda")
    yA16 = torch.empty(n, h, w, c1, dtype=torch.bfloat16, device="cuda")
    yA16g = torch.empty_like(yA16)
    yA32 = torch.empty(n, h, w, c1, device="cuda")
    fwd = lambda o: call("of_conv2d_b16i", 0, C.byref(dA), C.byref(o), P(wfA), P(bias), None,
                         None, None, None, 0.0, ACT_LEAKY, 0.3, st)
    fwd(io(a16=x16, lda16=l0, y16=yA16, ldy16=c1, mask_out=mask))          # direct
    fwd(io(a16=x16, lda16=l0, y=yA32, ldy=c1))                             # general, fp32
    assert lib.of_set_tuning(22, 0) == 0
    try:
        fwd(io(a16=x16, lda16=l0, y16=yA16g, ldy16=c1))                    # general, bf16
    finally:
        lib.of_set_tuning(22, 1)
    tiles = lib.of_conv2d_b16i_tiles(1, C.byref(dB))
    parts = [torch.empty(tiles, c1, device="cuda") for _ in range(2)]
    dbs = [torch.empty(c1, device="cuda") for _ in range(2)]
    gx = [torch.empty(n, h, w, c1, dtype=torch.bfloat16, device="cuda") for _ in range(2)]
    dgrad = lambda o: call("of_conv2d_b16i", 1, C.byref(dB), C.byref(o), P(wbB), None, None, None,
                           None, None, 0.0, ACT_LEAKY, 0.3, st)
    dgrad(io(a16=dy16, lda16=l2, y16=gx[0], ldy16=c1, mask_in=mask, col_part=parts[0]))
    dgrad(io(a16=dy16, lda16=l2, y16=gx[1], ldy16=c1, act_src=yA32, ld_act=c1, col_part=parts[1]))
    for k in range(2):
        call("of_col_part_reduce", P(parts[k]), tiles, c1, P(dbs[k]), 0, st)
    torch.cuda.synchronize()
    assert torch.equal(yA16, yA16g), "direct forward image != the general epilogue's"
    assert torch.equal(yA16, yA32.bfloat16()), "forward image != RNE of the fp32 output"
    assert torch.equal(gx[0], gx[1]), "mask_in input gradient != act_src input gradient"
    assert rel_l2(dbs[0], dbs[1]) < 1e-6, "column sums"


@pytest.mark.parametrize("n,h,w", [(2, 64, 96), (1, 50, 70), (3, 38, 130), (8, 384, 512)])
def test_conv_stem_b16(n, h, w):
    """The bf16 stem (configs 3-5) on the one-plane stem kernels (conv_stem_x3<32, 1>,
    conv_wgrad_stem_x3<1>; of_set_tuning key 15 = 1) against the bf16 implicit GEMMs (key 15
    = 0) and the float64 oracle on bf16-rounded operands: forward with bias, BN and ReLU in the
    epilogue, weight and bias gradients with accumulate, ragged tiles and the bench's B = 32
    image size (B = 8 here); the timing kinds say which kernels
    ran."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_RELU, call
    lib = _lib.lib()
    cin, cout = 4, 64
    xc = rng_tensor((n, h, w, 3), 81)
    x = torch.cat([xc, torch.zeros(n, h, w, 1)], -1)
    wt = rng_tensor((7, 7, 3, cout), 82, scale=(2.0 / 147) ** 0.5)
    b = rng_tensor((cout,), 83, scale=0.1)
    g, be = rng_tensor((cout,), 84, scale=0.5) + 1.0, rng_tensor((cout,), 85, scale=0.1)
    mu, var = rng_tensor((cout,), 86, scale=0.1), rng_tensor((cout,), 87).abs() + 0.5
    layer = ops.ConvLayer(dev(wt), dev(b), stride=2, act=ACT_RELU, cin_p=cin, precision="bf16")
    assert layer.bf16()
    d = layer.desc(n, h, w)
    dz = rng_tensor((n, d.ho, d.wo, cout), 88)
    wf, _ = layer.packed(d)
    fent, fws = layer.fwd_entry(d)
    went, _ = layer.wgrad_entry(d)
    ws = torch.empty(fws // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    xd, bd, gd, bed, mud, vard, dzd = [dev(t) for t in (x, b, g, be, mu, var, dz)]
    prior_w, prior_b = rng_tensor((7, 7, 3, cout), 89), rng_tensor((cout,), 90)

    def kinds():
        kk = (C.c_int * 16)()
        cnt = lib.of_timing_read(16, kk, None, None)
        return {kk[i] for i in range(cnt)}

    res = {}
    try:
        for form in (1, 0):
            assert lib.of_set_tuning(15, form) == 0
            y = torch.full((n, d.ho, d.wo, cout), 7.0, device="cuda")
            lib.of_timing_enable(1)
            call(fent, C.byref(d), P(xd), cin, P(wf), P(bd), P(gd), P(bed), P(mud), P(vard), 1e-3,
                 None, 0, ACT_RELU, 0.0, None, 0, P(y), cout, P(ws), fws, st)
            torch.cuda.synchronize()
            kf = kinds()
            wws = getattr(lib, went + "_workspace")(C.byref(d))
            wsw = torch.empty(wws // 4 + 4, device="cuda")
            dw, db = dev(prior_w.clone()), dev(prior_b.clone())
            call(went, C.byref(d), P(xd), cin, P(dzd), cout, P(dw), P(db), 1, P(wsw), wws, st)
            torch.cuda.synchronize()
            kw = kinds()
            lib.of_timing_enable(0)
            res[form] = (y, dw.cpu().double() - f64(prior_w), db.cpu().double() - f64(prior_b),
                         kf, kw)
    finally:
        lib.of_set_tuning(15, 1)
        lib.of_timing_enable(0)
    assert res[1][3] == {186} and 186 not in res[0][3], (res[1][3], res[0][3])
    assert res[1][4] == {187} and 187 not in res[0][4], (res[1][4], res[0][4])
    # oracle: bf16-rounded x and w, float64 arithmetic, BN + ReLU on the fp64 sum
    zref = R._Bf16Conv.apply(f64(xc), f64(wt), f64(b), 2)
    yref = torch.relu((zref - f64(mu)) / torch.sqrt(f64(var) + 1e-3) * f64(g) + f64(be))
    wo = f64(wt).requires_grad_(True)
    (R._Bf16Conv.apply(f64(xc), wo, None, 2) * f64(dz)).sum().backward()
    dbref = f64(dz).sum((0, 1, 2))
    for form in (1, 0):
        y, dwv, dbv = res[form][:3]
        assert rel_inf(y, yref) < REL_TOL, (form, rel_inf(y, yref))
        assert rel_l2(dwv, wo.grad) < REL_TOL, (form, rel_l2(dwv, wo.grad))
        assert rel_l2(dbv, dbref) < 1e-5, (form, rel_l2(dbv, dbref))
    # the two kernel families differ only in fp32 summation order
    assert rel_inf(res[1][0], res[0][0]) < 1e-5
    assert rel_l2(res[1][1], res[0][1]) < 1e-5


@pytest.mark.parametrize("n,h,w", [(2, 64, 96), (1, 50, 70), (3, 38, 130), (8, 384, 512)])
def test_conv_stem_wgrad_x3(n, h, w):
    """The stem's weight gradient on its own split-bf16 kernel (conv_wgrad_stem_x3: 4 x 32
    output tiles, the input halo split by column parity in LDS, persistent workgroups, one
    slab each) against fp64 and against the fp32 MFMA GEMM (of_set_tuning key 14 = 0): the
    kernel and bias gradients, accumulate, ragged tiles, and the bench's full size (B = 8,
    384 x 512); as accurate as one fp32 rounding per product; the timing kind says which
    kernel ran."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_RELU, call
    lib = _lib.lib()
    cin, cout = 4, 64
    xc = rng_tensor((n, h, w, 3), 71)
    x = torch.cat([xc, torch.zeros(n, h, w, 1)], -1)
    wt = rng_tensor((7, 7, 3, cout), 72, scale=(2.0 / 147) ** 0.5)
    layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=2, act=ACT_RELU, cin_p=cin,
                          f32_split=True)
    d = layer.desc(n, h, w)
    dz = rng_tensor((n, d.ho, d.wo, cout), 73)
    went, _ = layer.wgrad_entry(d)
    xd, dzd = dev(x), dev(dz)
    P, st = ops._ptr, ops._stream()
    prior_w = rng_tensor((7, 7, 3, cout), 74)
    prior_b = rng_tensor((cout,), 75)
    res = {}
    try:
        for form in (1, 0):
            assert lib.of_set_tuning(14, form) == 0
            wws = getattr(lib, went + "_workspace")(C.byref(d))
            ws = torch.empty(wws // 4 + 4, device="cuda")
            dw, db = dev(prior_w.clone()), dev(prior_b.clone())
            lib.of_timing_enable(1)
            call(went, C.byref(d), P(xd), cin, P(dzd), cout, P(dw), P(db), 1, P(ws), wws, st)
            torch.cuda.synchronize()
            lib.of_timing_enable(0)
            kk = (C.c_int * 16)()
            cnt = lib.of_timing_read(16, kk, None, None)
            res[form] = (dw.cpu().double() - f64(prior_w), db.cpu().double() - f64(prior_b),
                         {kk[i] for i in range(cnt)})
    finally:
        lib.of_set_tuning(14, 1)
        lib.of_timing_enable(0)
    assert res[1][2] == {185} and 185 not in res[0][2], (res[1][2], res[0][2])
    wo = f64(wt).requires_grad_(True)
    (R.conv2d_same(f64(xc), wo, None, 2) * f64(dz)).sum().backward()
    dbref = f64(dz).sum((0, 1, 2))
    e_new = [rel_l2(res[1][0], wo.grad), rel_l2(res[1][1], dbref)]
    e_old = [rel_l2(res[0][0], wo.grad), rel_l2(res[0][1], dbref)]
    print("stem wgrad rel_l2 new %s, fp32 GEMM %s" % (e_new, e_old))
    # (the accumulate subtraction leaves fp32 rounding of the prior values: 1e-6 relative)
    assert e_new[0] < 3 * e_old[0] + 1e-6 and e_new[0] < 5e-6, (e_new, e_old)
    assert e_new[1] < 5e-6, (e_new, e_old)


@pytest.mark.parametrize("case,n,h,w,cin,cout,kinds", [
    # kinds: 128 + 8 mode + cfg; wgrad 144 + cfg (3-tap form) / 148 + cfg (9-tap x3b form)
    ("tall128", 8, 128, 256, 128, 128, {128, 136, 148}),  # 8 x 32 tiles, BN 128 (1024 tiles)
    ("tall96", 8, 128, 256, 128, 96, {133, 136, 145}),    # 8 x 32 tiles, BN 96 fwd; BN 128 dgrad
    ("nb1", 8, 64, 128, 128, 128, {132, 140, 148}),       # single-buffered two-per-CU 4 x 32 form
    ("split", 2, 48, 64, 256, 256, {134, 142, 148}),      # 8-wave 4 x 32 form with a K split
    ("split64", 2, 48, 64, 256, 256, {130, 138, 148}),    # small grid: BN 64 tiles (key 27)
    ("bn64", 8, 128, 256, 64, 64, {130, 138, 146}),       # BN 64 keeps 4 x 32 tiles on large grids
], ids=["tall128", "tall96", "nb1", "split", "split64", "bn64"])
def test_conv_x3_large_grids(case, n, h, w, cin, cout, kinds):
    """The grid-size-selected forms of the split kernels (taller output tiles, the
    single-buffered two-workgroups-per-CU form, K splits) against the fp32 MFMA kernels on
    the same inputs, with the fused LeakyReLU / bias (fwd) and activation-derivative (dgrad)
    epilogues and the weight + bias gradient; both paths are checked against the oracle
    elsewhere, so agreement within fp32 accumulation-order noise pins these forms."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd._lib import ACT_LEAKY, call
    x = dev(rng_tensor((n, h, w, cin), 31))
    wt = dev(rng_tensor((3, 3, cin, cout), 32, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 33, scale=0.1))
    dy = dev(rng_tensor((n, h, w, cout), 34))
    act_src = dev(rng_tensor((n, h, w, cin), 35))
    from optical_flow_amd import _lib
    lib = _lib.lib()
    outs = {}
    lib.of_timing_read(0, None, None, None)          # drop records of earlier launches
    if case in ("split", "nb1"):                     # the BN = 128 forms (key 27 off)
        assert lib.of_set_tuning(27, 0) == 0
    try:
        _large_grid_forms(ops, lib, case, n, h, w, cin, cout, kinds, x, wt, b, dy, act_src, outs)
    finally:
        lib.of_set_tuning(27, 1200)                  # (the default, conv_f32.hip)
    for name, a3, a32 in zip(("y", "dx", "dw", "db"), outs[True], outs[False]):
        assert rel_inf(a3, a32) < 2e-5, name
        assert rel_l2(a3, a32) < 5e-6, name


def _large_grid_forms(ops, lib, case, n, h, w, cin, cout, kinds, x, wt, b, dy, act_src, outs):
    import ctypes as C
    from optical_flow_amd._lib import ACT_LEAKY, call
    for split in (True, False):
        lib.of_timing_enable(1 if split else 0)
        layer = ops.ConvLayer(wt, b, stride=1, act=ACT_LEAKY, cin_p=cin, f32_split=split)
        d = layer.desc(n, h, w)
        assert layer.mode(d) == (2 if split else 0)
        wf, wd = layer.packed(d)
        fent, fws = layer.fwd_entry(d)
        dent, dws = layer.dgrad_entry(d)
        went, wws = layer.wgrad_entry(d)
        if split:
            # the fwd / dgrad workspace holds the K-split slabs: nonzero exactly when the plan
            # splits K, so this pins the split / unsplit forms each case is meant to cover
            if case in ("split", "split64"):
                assert fws > 0 and dws > 0, (fws, dws)
            else:
                assert fws == 0 and dws == 0, (fws, dws)
        ws = torch.empty(max(fws, dws, wws) // 4 + 4, device="cuda")
        P, st = ops._ptr, ops._stream()
        y = torch.empty(n, h, w, cout, device="cuda")
        dx = torch.empty(n, h, w, cin, device="cuda")
        dw = torch.empty_like(wt)
        db = torch.empty_like(b)
        call(fent, C.byref(d), P(x), cin, P(wf), P(b), None, None, None, None, 1e-3, None, 0,
             ACT_LEAKY, 0.3, None, 0, P(y), cout, P(ws), fws, st)
        call(dent, C.byref(d), P(dy), cout, P(wd), P(act_src), cin, ACT_LEAKY, 0.3, P(dx), cin,
             P(ws), dws, st)
        call(went, C.byref(d), P(x), cin, P(dy), cout, P(dw), P(db), 0, P(ws), wws, st)
        torch.cuda.synchronize()
        if split:    # the timing kinds name the kernel configurations that ran (bench.py)
            lib.of_timing_enable(0)
            cap = 64
            k_arr, f_arr, m_arr = (C.c_int * cap)(), (C.c_double * cap)(), (C.c_float * cap)()
            got = {k_arr[i] for i in range(lib.of_timing_read(cap, k_arr, f_arr, m_arr))}
            assert kinds <= got, (kinds, got)
        outs[split] = (y, dx, dw, db)


@pytest.mark.parametrize("case,n,h,w,cin,cout,kinds", [
    # kinds: 224 + 8 mode + cfg (cfg 0: BN 128, 1: BN 96; family tile_ws)
    ("tall128", 8, 128, 256, 128, 128, {224, 232}),
    ("tall96", 8, 128, 256, 128, 96, {225, 232}),
    ("split", 2, 48, 64, 256, 256, {224, 232}),      # K split over channel chunks
    ("ragged", 2, 41, 70, 128, 128, {224, 232}),     # partial tiles at the image border
    ("c0", 2, 48, 64, 120, 96, {225, 232}),          # concat row: a partial channel chunk
    ("single", 1, 8, 32, 32, 128, {224}),            # fwd one chunk: 9 steps (dgrad N 32: not ws)
], ids=["tall128", "tall96", "split", "ragged", "c0", "single"])
def test_conv_ws_forms(case, n, h, w, cin, cout, kinds):
    """bf16 fwd / dgrad on the warp-specialised conv_tile_ws (of_set_tuning key 12 = 2)
    against the round-1 conv_tile_bf16 (key 12 = 0) on the same inputs: both round x, dy and
    the weights to bf16 RNE and accumulate in fp32, so they agree to accumulation-order noise;
    the timing kinds name the configurations that ran.  test_conv_bf16 checks the default
    kernels against the oracle."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, call
    lib = _lib.lib()
    x = dev(rng_tensor((n, h, w, cin), 61))
    wt = dev(rng_tensor((3, 3, cin, cout), 62, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 63, scale=0.1))
    dy = dev(rng_tensor((n, h, w, cout), 64))
    act_src = dev(rng_tensor((n, h, w, cin), 65))
    outs = {}
    lib.of_timing_read(0, None, None, None)
    try:
        for form in (2, 0):
            assert lib.of_set_tuning(12, form) == 0
            lib.of_timing_enable(1 if form else 0)
            layer = ops.ConvLayer(wt, b, stride=1, act=ACT_LEAKY, cin_p=cin, precision="bf16")
            d = layer.desc(n, h, w)
            assert layer.bf16(d)
            wf, wd = layer.packed(d)
            fent, fws = layer.fwd_entry(d)
            dent, dws = layer.dgrad_entry(d)
            if case == "split" and form:
                assert fws > 0 and dws > 0, (fws, dws)
            ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
            P, st = ops._ptr, ops._stream()
            y = torch.empty(n, h, w, cout, device="cuda")
            dx = torch.empty(n, h, w, cin, device="cuda")
            call(fent, C.byref(d), P(x), cin, P(wf), P(b), None, None, None, None, 1e-3, None, 0,
                 ACT_LEAKY, 0.3, None, 0, P(y), cout, P(ws), fws, st)
            call(dent, C.byref(d), P(dy), cout, P(wd), P(act_src), cin, ACT_LEAKY, 0.3, P(dx),
                 cin, P(ws), dws, st)
            torch.cuda.synchronize()
            if form:
                lib.of_timing_enable(0)
                cap = 64
                k_arr, f_arr, m_arr = (C.c_int * cap)(), (C.c_double * cap)(), (C.c_float * cap)()
                got = {k_arr[i] for i in range(lib.of_timing_read(cap, k_arr, f_arr, m_arr))}
                assert kinds <= got, (kinds, got)
            outs[form] = (y, dx)
    finally:
        lib.of_set_tuning(12, 0)                    # the default
        lib.of_timing_enable(0)
    for name, a1, a0 in zip(("y", "dx"), outs[2], outs[0]):
        e = rel_l2(a1, a0)
        print("%s %s rel_l2 %.2e rel_inf %.2e" % (case, name, e, rel_inf(a1, a0)))
        assert e < 1e-5 and rel_inf(a1, a0) < 1e-4, name


@pytest.mark.parametrize("case,n,h,w,cin,cout,kinds", [
    # kinds: 192 + 8 mode + cfg (bench.py kind_parts, family tile_b16)
    ("tall128", 8, 128, 256, 128, 128, {192, 200, 216}),   # 8 x 32 tiles, BN 128 (1024 tiles)
    ("tall96", 8, 128, 256, 128, 96, {197, 200, 217}),     # 8 x 32 tiles, BN 96 fwd; BN 128 dgrad
    ("bn128", 8, 64, 128, 128, 128, {198, 206, 216}),      # 4 x 32 tiles, 8 waves, two WGs per CU
    ("split", 2, 48, 64, 256, 256, {198, 206, 216}),       # K split over channel chunks
    ("bn64", 8, 128, 256, 64, 64, {194, 202, 218}),        # BN 64
    ("bn32", 2, 40, 70, 32, 32, {195, 203, 219}),          # BN 32, ragged
    ("c0", 2, 48, 64, 120, 96, {193, 206, 217}),           # concat row (120 ch: a partial chunk)
    ("c3", 2, 48, 64, 96, 64, {194, 201, 220}),            # 96 -> 64: wgrad 32 x 64 blocks
], ids=["tall128", "tall96", "bn128", "split", "bn64", "bn32", "c0", "c3"])
def test_conv_b16_forms(case, n, h, w, cin, cout, kinds):
    """bf16 fwd / dgrad on conv_tile_b16 and the weight gradient on conv_wgrad_tile_b16 (the
    split kernels' structures with one plane) against the round-1 conv_tile_bf16 /
    conv_wgrad_tile_bf16 (of_set_tuning keys 12, 13 = 0) on the same inputs: both round x, dy
    and the weights to bf16 RNE and accumulate in fp32, so they agree to accumulation-order
    noise (measured: bitwise equal but for the bias column sums); the timing kinds name the
    configurations that ran.  test_conv_bf16 checks the default kernels against the oracle."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, call
    lib = _lib.lib()
    x = dev(rng_tensor((n, h, w, cin), 51))
    wt = dev(rng_tensor((3, 3, cin, cout), 52, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 53, scale=0.1))
    dy = dev(rng_tensor((n, h, w, cout), 54))
    act_src = dev(rng_tensor((n, h, w, cin), 55))
    outs = {}
    lib.of_timing_read(0, None, None, None)
    try:
        for form in (1, 0):
            assert lib.of_set_tuning(12, form) == 0
            assert lib.of_set_tuning(13, form) == 0
            lib.of_timing_enable(1 if form else 0)
            layer = ops.ConvLayer(wt, b, stride=1, act=ACT_LEAKY, cin_p=cin, precision="bf16")
            d = layer.desc(n, h, w)
            assert layer.bf16(d)
            wf, wd = layer.packed(d)
            fent, fws = layer.fwd_entry(d)
            dent, dws = layer.dgrad_entry(d)
            went, wws = layer.wgrad_entry(d)
            if case == "split" and form:
                assert fws > 0 and dws > 0, (fws, dws)
            ws = torch.empty(max(fws, dws, wws) // 4 + 4, device="cuda")
            P, st = ops._ptr, ops._stream()
            y = torch.empty(n, h, w, cout, device="cuda")
            dx = torch.empty(n, h, w, cin, device="cuda")
            call(fent, C.byref(d), P(x), cin, P(wf), P(b), None, None, None, None, 1e-3, None, 0,
                 ACT_LEAKY, 0.3, None, 0, P(y), cout, P(ws), fws, st)
            call(dent, C.byref(d), P(dy), cout, P(wd), P(act_src), cin, ACT_LEAKY, 0.3, P(dx),
                 cin, P(ws), dws, st)
            dw = torch.empty_like(wt)
            db = torch.empty_like(b)
            call(went, C.byref(d), P(x), cin, P(dy), cout, P(dw), P(db), 0, P(ws), wws, st)
            torch.cuda.synchronize()
            if form:
                lib.of_timing_enable(0)
                cap = 64
                k_arr, f_arr, m_arr = (C.c_int * cap)(), (C.c_double * cap)(), (C.c_float * cap)()
                got = {k_arr[i] for i in range(lib.of_timing_read(cap, k_arr, f_arr, m_arr))}
                assert kinds <= got, (kinds, got)
            outs[form] = (y, dx, dw, db)
    finally:
        lib.of_set_tuning(12, 0)                    # the defaults
        lib.of_set_tuning(13, 0)
        lib.of_timing_enable(0)
    for name, a1, a0 in zip(("y", "dx", "dw", "db"), outs[1], outs[0]):
        e = rel_l2(a1, a0)
        print("%s %s rel_l2 %.2e rel_inf %.2e" % (case, name, e, rel_inf(a1, a0)))
        assert e < 1e-5 and rel_inf(a1, a0) < 1e-4, name


@pytest.mark.parametrize("n,h,w,cin,cout", [
    (2, 20, 45, 64, 128),     # ragged right edge (45 px), 4 x 32 tiles
    (8, 128, 256, 128, 128),  # 8 x 32 tiles, BN 128
    (2, 48, 64, 256, 256),    # K split: the epilogue writes slab rows
    (2, 16, 24, 64, 96),      # BN 96
    (3, 9, 40, 32, 64),       # BN 64, odd rows
    (2, 8, 40, 32, 32),       # BN 32
    (1, 6, 10, 256, 44),      # N % 4 == 0 but not a tile multiple
    (1, 6, 10, 64, 42),       # N % 4 != 0: per-element epilogue either way
])
def test_conv_x3_vec_epilogue(n, h, w, cin, cout):
    """The split kernels' 16-byte epilogue (accumulators transposed through LDS, float4
    columns) is bitwise identical to the per-element one (of_set_tuning key 3): fwd with bias,
    BN, the residual, z and ReLU; dgrad with the activation derivative and an added gradient."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, ACT_RELU, call
    lib = _lib.lib()
    x = dev(rng_tensor((n, h, w, cin), 41))
    wt = dev(rng_tensor((3, 3, cin, cout), 42, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 43, scale=0.1))
    g, be = dev(rng_tensor((cout,), 44, scale=0.5)) + 1.0, dev(rng_tensor((cout,), 45, scale=0.1))
    mu, var = dev(rng_tensor((cout,), 46, scale=0.1)), dev(rng_tensor((cout,), 47)).abs() + 0.5
    coutp = (cout + 3) // 4 * 4
    res = dev(rng_tensor((n, h, w, cout), 48))
    dy = dev(rng_tensor((n, h, w, coutp), 49))
    act_src = dev(rng_tensor((n, h, w, cin), 50))
    add = dev(rng_tensor((n, h, w, cin), 51))
    layer = ops.ConvLayer(wt, b, stride=1, act=ACT_RELU, cin_p=cin, f32_split=True)
    d = layer.desc(n, h, w)
    assert layer.mode(d) == 2
    wf, wd = layer.packed(d)
    fent, fws = layer.fwd_entry(d)
    dws = lib.of_conv2d_dgrad_x3_workspace(C.byref(d))
    ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    outs = []
    try:
        for vec in (1, 0):
            assert lib.of_set_tuning(3, vec) == 0
            y = torch.full((n, h, w, cout), 7.0, device="cuda")
            z = torch.full((n, h, w, cout), 7.0, device="cuda")
            dx = torch.full((n, h, w, cin), 7.0, device="cuda")
            dx2 = torch.full((n, h, w, cin), 7.0, device="cuda")
            call(fent, C.byref(d), P(x), cin, P(wf), P(b), P(g), P(be), P(mu), P(var), 1e-3,
                 P(res), cout, ACT_RELU, 0.0, P(z), cout, P(y), cout, P(ws), fws, st)
            call("of_conv2d_dgrad_x3", C.byref(d), P(dy), coutp, P(wd), P(act_src), cin,
                 ACT_LEAKY, 0.3, P(dx), cin, P(ws), dws, st)
            call("of_conv2d_dgrad_add_x3", C.byref(d), P(dy), coutp, P(wd), P(add), cin,
                 P(dx2), cin, P(ws), dws, st)
            torch.cuda.synchronize()
            outs.append((y, z, dx, dx2))
    finally:
        lib.of_set_tuning(3, 1)
    for name, a1, a0 in zip(("y", "z", "dx", "dx_add"), *outs):
        assert torch.equal(a1, a0), (name, (a1 - a0).abs().max().item())
    yref = torch.relu((R.conv2d_same(f64(x), f64(wt), f64(b), 1) - f64(mu)) / torch.sqrt(f64(var) + 1e-3)
                      * f64(g) + f64(be) + f64(res))
    assert rel_inf(outs[0][0], yref) < REL_TOL


@pytest.mark.parametrize("n,h,w,cin,cout", [
    (8, 128, 256, 128, 128),  # 8-wave <128, 4, 2> dgrad, 8 x 32 tiles
    (4, 67, 250, 96, 128),    # ragged bottom / right edges
    (8, 64, 128, 96, 96),     # BN 96, 12 waves
])
def test_conv_x3_direct_dgrad(n, h, w, cin, cout):
    """The split input gradient's direct epilogue (of_set_tuning key 23 bit 1, off by default:
    row image + whole 16-byte chunks with the activation-source / added-gradient quads loaded
    ahead) is bitwise the per-pass transposes' result: activation derivative, added gradient, and the
    added gradient in place."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, call
    lib = _lib.lib()
    wt = dev(rng_tensor((3, 3, cin, cout), 52, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 53, scale=0.1))
    dy = dev(rng_tensor((n, h, w, cout), 54))
    act_src = dev(rng_tensor((n, h, w, cin), 55))
    add = dev(rng_tensor((n, h, w, cin), 56))
    layer = ops.ConvLayer(wt, b, stride=1, act=ACT_LEAKY, cin_p=cin, f32_split=True)
    d = layer.desc(n, h, w)
    assert layer.mode(d) == 2
    _, wd = layer.packed(d)
    dws = lib.of_conv2d_dgrad_x3_workspace(C.byref(d))
    assert dws == 0                       # one K slice: the direct epilogue's precondition
    P, st = ops._ptr, ops._stream()
    outs = []
    try:
        for key in (3, 1):
            assert lib.of_set_tuning(23, key) == 0
            dx = torch.full((n, h, w, cin), 7.0, device="cuda")
            dx2 = torch.full((n, h, w, cin), 7.0, device="cuda")
            dx3 = add.clone()
            call("of_conv2d_dgrad_x3", C.byref(d), P(dy), cout, P(wd), P(act_src), cin,
                 ACT_LEAKY, 0.3, P(dx), cin, None, 0, st)
            call("of_conv2d_dgrad_add_x3", C.byref(d), P(dy), cout, P(wd), P(add), cin,
                 P(dx2), cin, None, 0, st)
            call("of_conv2d_dgrad_add_x3", C.byref(d), P(dy), cout, P(wd), P(dx3), cin,
                 P(dx3), cin, None, 0, st)
            torch.cuda.synchronize()
            outs.append((dx, dx2, dx3))
    finally:
        lib.of_set_tuning(23, 1)
    for name, a1, a0 in zip(("dx", "dx_add", "dx_add_in_place"), *outs):
        assert torch.equal(a1, a0), (name, (a1 - a0).abs().max().item())
    assert torch.equal(outs[0][1], outs[0][2])
    # (the per-pass form is pinned against fp64 by test_conv_x3_large_grids / _accuracy)


@pytest.mark.parametrize("n,h,w,cin,cout", [
    (2, 20, 45, 128, 128),   # <2,4,8>: ragged right edge, 2 channel tiles
    (1, 13, 32, 64, 96),     # <2,3,8>: odd rows (half k-step at the bottom)
    (2, 24, 32, 64, 64),     # <4,2,4>
    (1, 9, 40, 64, 32),      # <4,1,4>
    (2, 8, 16, 256, 256),    # deep split over tiles, 16 channel tiles
    (1, 6, 10, 44, 128),     # cin 44: partial channel block
])
def test_wgrad_x3_forms(n, h, w, cin, cout):
    """The 9-tap split-bf16 weight gradient (conv_wgrad_tile_x3b: of_set_tuning key 4 = 2
    runs it for every Cout) against fp64 and against the 3-tap form (key 4 = 0): weights and
    bias gradient, with the 16-byte slab epilogue and the per-element one."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_NONE, call
    lib = _lib.lib()
    x = dev(rng_tensor((n, h, w, cin), 81))
    wt = dev(rng_tensor((3, 3, cin, cout), 82, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 83, scale=0.1))
    coutp = (cout + 3) // 4 * 4
    dy = dev(rng_tensor((n, h, w, coutp), 84))
    layer = ops.ConvLayer(wt, b, stride=1, act=ACT_NONE, cin_p=cin, f32_split=True)
    d = layer.desc(n, h, w)
    wws = lib.of_conv2d_wgrad_x3_workspace(C.byref(d))
    ws = torch.empty(wws // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    dwref = torch.nn.grad.conv2d_weight(f64(x).permute(0, 3, 1, 2), (cout, cin, 3, 3),
                                        f64(dy[..., :cout]).permute(0, 3, 1, 2),
                                        padding=1).permute(2, 3, 1, 0)
    dbref = f64(dy[..., :cout]).sum((0, 1, 2))
    outs = {}
    try:
        for form, vec in ((2, 1), (2, 0), (0, 1)):
            assert lib.of_set_tuning(4, form) == 0 and lib.of_set_tuning(3, vec) == 0
            dw = torch.full_like(wt, 7.0)
            db = torch.full_like(b, 7.0)
            call("of_conv2d_wgrad_x3", C.byref(d), P(x), cin, P(dy), coutp, P(dw), P(db), 0,
                 P(ws), wws, st)
            torch.cuda.synchronize()
            outs[(form, vec)] = (dw, db)
    finally:
        lib.of_set_tuning(4, 1)
        lib.of_set_tuning(3, 1)
    assert torch.equal(outs[(2, 1)][0], outs[(2, 0)][0]) and torch.equal(outs[(2, 1)][1], outs[(2, 0)][1])
    for key, (dw, db) in outs.items():
        assert rel_inf(dw, dwref) < 5e-6, (key, rel_inf(dw, dwref))
        assert rel_inf(db, dbref) < 5e-6, (key, rel_inf(db, dbref))


@pytest.mark.parametrize("n,h,w,cin", [(2, 24, 32, 96), (1, 13, 40, 32), (1, 9, 20, 160)])
def test_wgrad_x3_cout64_32ci_blocks(n, h, w, cin):
    """Cout 64 with Cin not a multiple of 64 (the 96 -> 64 flow-head convs): the 9-tap split
    weight gradient on 32 x 64 channel blocks (cfg 4, of_set_tuning key 11 = 1, timing kind
    152) against fp64 and against the 64 x 64 blocks (key 11 = 0; odd rows, ragged columns)."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_NONE, call
    lib = _lib.lib()
    cout = 64
    x = dev(rng_tensor((n, h, w, cin), 91))
    wt = dev(rng_tensor((3, 3, cin, cout), 92, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 93, scale=0.1))
    dy = dev(rng_tensor((n, h, w, cout), 94))
    layer = ops.ConvLayer(wt, b, stride=1, act=ACT_NONE, cin_p=cin, f32_split=True)
    d = layer.desc(n, h, w)
    P, st = ops._ptr, ops._stream()
    dwref = torch.nn.grad.conv2d_weight(f64(x).permute(0, 3, 1, 2), (cout, cin, 3, 3),
                                        f64(dy).permute(0, 3, 1, 2), padding=1).permute(2, 3, 1, 0)
    dbref = f64(dy).sum((0, 1, 2))
    outs = {}
    k_arr = (C.c_int * 8)()
    try:
        for c4 in (1, 0):
            assert lib.of_set_tuning(11, c4) == 0
            wws = lib.of_conv2d_wgrad_x3_workspace(C.byref(d))
            ws = torch.empty(wws // 4 + 4, device="cuda")
            dw = torch.full_like(wt, 7.0)
            db = torch.full_like(b, 7.0)
            lib.of_timing_read(0, None, None, None)
            lib.of_timing_enable(1)
            call("of_conv2d_wgrad_x3", C.byref(d), P(x), cin, P(dy), cout, P(dw), P(db), 0,
                 P(ws), wws, st)
            torch.cuda.synchronize()
            lib.of_timing_enable(0)
            kinds = {k_arr[i] for i in range(lib.of_timing_read(8, k_arr, None, None))}
            assert kinds == ({152} if c4 else {146}), (c4, kinds)
            outs[c4] = (dw, db)
    finally:
        lib.of_set_tuning(11, 1)
        lib.of_timing_enable(0)
    for key, (dw, db) in outs.items():
        assert rel_inf(dw, dwref) < 5e-6, (key, rel_inf(dw, dwref))
        assert rel_inf(db, dbref) < 5e-6, (key, rel_inf(db, dbref))


@pytest.mark.parametrize("prec", ["f32", "bf16", "x3"])
@pytest.mark.parametrize("n,h,w,cin,cout,k,s", [
    (2, 32, 48, 4, 64, 7, 2),      # stem: 256 x 64 tiles, split-K slabs
    (2, 16, 24, 64, 128, 3, 2),    # stride-2 block conv: dgrad phase groups
    (2, 16, 24, 64, 128, 1, 2),    # 1x1 projection: in-place dgrad add skips 3 phase groups
    (2, 12, 20, 128, 96, 3, 1),    # f32: 128 x 96 tiles; bf16: halo tiles
    (1, 6, 10, 64, 36, 3, 1),      # 256 x 64 tiles, N not a tile multiple
    (2, 20, 45, 128, 128, 3, 1),   # bf16 halo tiles, ragged right edge
])
def test_conv_gemm_vec_epilogue(n, h, w, cin, cout, k, s, prec, monkeypatch):
    """The fp32 / bf16 / split-bf16 (x3) implicit-GEMM and the halo-tile kernels' 16-byte
    epilogues are bitwise identical to the per-element one: fwd (bias, BN, residual, z,
    ReLU), dgrad (activation derivative; added gradient, in place), wgrad slabs + bias sums."""
    import ctypes as C
    ops = _ops()
    monkeypatch.setattr(ops, "X3_GEMM_MIN_CIN", 0)   # the stem shape on conv_gemm_x3 too
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, ACT_RELU, call
    lib = _lib.lib()
    x = dev(rng_tensor((n, h, w, cin), 61))
    wt = dev(rng_tensor((k, k, cin, cout), 62, scale=(2.0 / (k * k * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 63, scale=0.1))
    g, be = dev(rng_tensor((cout,), 64, scale=0.5)) + 1.0, dev(rng_tensor((cout,), 65, scale=0.1))
    mu, var = dev(rng_tensor((cout,), 66, scale=0.1)), dev(rng_tensor((cout,), 67)).abs() + 0.5
    if prec == "bf16":
        layer = ops.ConvLayer(wt, b, stride=s, act=ACT_RELU, cin_p=cin, precision="bf16")
    else:
        layer = ops.ConvLayer(wt, b, stride=s, act=ACT_RELU, cin_p=cin, f32_split=prec == "x3")
    d = layer.desc(n, h, w)
    sfx = {"bf16": "_bf16", "x3": "_x3", "f32": ""}[prec]
    assert layer.mode(d) == {"f32": 0, "bf16": 1, "x3": 2}[prec]
    ho, wo = d.ho, d.wo
    coutp = (cout + 3) // 4 * 4
    res = dev(rng_tensor((n, ho, wo, cout), 68))
    dy = dev(rng_tensor((n, ho, wo, coutp), 69))
    act_src = dev(rng_tensor((n, h, w, cin), 70))
    add = dev(rng_tensor((n, h, w, cin), 71))
    wf, wd = layer.packed(d)
    # the stem shape: conv_gemm_x3 in both arms (conv_stem_x3 has the 16-byte epilogue only;
    # test_conv_stem_x3 covers it), of_set_tuning key 8 restored below
    assert lib.of_set_tuning(8, 0) == 0
    fws = getattr(lib, "of_conv2d_fwd%s_workspace" % sfx)(C.byref(d))
    dws = getattr(lib, "of_conv2d_dgrad%s_workspace" % sfx)(C.byref(d))
    wws = getattr(lib, "of_conv2d_wgrad%s_workspace" % sfx)(C.byref(d))
    ws = torch.empty(max(fws, dws, wws) // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    outs = []
    try:
        for vec in (1, 0):
            assert lib.of_set_tuning(3, vec) == 0
            y = torch.full((n, ho, wo, cout), 7.0, device="cuda")
            z = torch.full((n, ho, wo, cout), 7.0, device="cuda")
            dx = torch.full((n, h, w, cin), 7.0, device="cuda")
            dx2 = add.clone()
            dw = torch.full_like(wt, 7.0)
            db = torch.full_like(b, 7.0)
            call("of_conv2d_fwd" + sfx, C.byref(d), P(x), cin, P(wf), P(b), P(g), P(be), P(mu),
                 P(var), 1e-3, P(res), cout, ACT_RELU, 0.0, P(z), cout, P(y), cout, P(ws), fws, st)
            if k < 7:
                call("of_conv2d_dgrad" + sfx, C.byref(d), P(dy), coutp, P(wd), P(act_src), cin,
                     ACT_LEAKY, 0.3, P(dx), cin, P(ws), dws, st)
                call("of_conv2d_dgrad_add" + sfx, C.byref(d), P(dy), coutp, P(wd), P(dx2), cin,
                     P(dx2), cin, P(ws), dws, st)
            call("of_conv2d_wgrad" + sfx, C.byref(d), P(x), cin, P(dy), coutp, P(dw), P(db), 0,
                 P(ws), wws, st)
            torch.cuda.synchronize()
            outs.append((y, z, dx, dx2, dw, db))
    finally:
        lib.of_set_tuning(3, 1)
        lib.of_set_tuning(8, 1)
    for name, a1, a0 in zip(("y", "z", "dx", "dx_add", "dw", "db"), *outs):
        assert torch.equal(a1, a0), (name, (a1 - a0).abs().max().item())
    zref = R.conv2d_same(f64(x), f64(wt), f64(b), s)
    assert rel_inf(outs[0][1], zref) < {"bf16": 2e-2, "f32": REL_TOL, "x3": 5e-6}[prec]
    if s == 1:
        dxref = torch.nn.grad.conv2d_input((n, cin, h, w), f64(wt).permute(3, 2, 0, 1),
                                           f64(dy[..., :cout]).permute(0, 3, 1, 2),
                                           padding=k // 2)
        assert rel_inf(outs[0][2], torch.where(f64(act_src) > 0, 1.0, 0.3) *
                       dxref.permute(0, 2, 3, 1)) < {"bf16": 2e-2, "f32": REL_TOL, "x3": 5e-6}[prec]


def test_conv_bf16_tall_fwd():
    """bf16 forward with 8 x 32 output tiles (grids of >= 1024 tiles, BN 128) against an fp64
    conv of the bf16-rounded operands (the bf16 kernels round x and w RNE while staging)."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_NONE, call
    lib = _lib.lib()
    n, h, w, cin, cout = 8, 128, 256, 128, 128
    x = rng_tensor((n, h, w, cin), 41)
    wt = rng_tensor((3, 3, cin, cout), 42, scale=(2.0 / (9 * cin)) ** 0.5)
    layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=1, act=ACT_NONE, cin_p=cin,
                          precision="bf16")
    d = layer.desc(n, h, w)
    wf, _ = layer.packed(d)
    fent, fws = layer.fwd_entry(d)
    ws = torch.empty(fws // 4 + 4, device="cuda")
    y = torch.empty(n, h, w, cout, device="cuda")
    lib.of_timing_read(0, None, None, None)
    lib.of_timing_enable(1)
    call(fent, C.byref(d), ops._ptr(dev(x)), cin, ops._ptr(wf), ops._ptr(layer.bias), None, None,
         None, None, 1e-3, None, 0, ACT_NONE, 0.0, None, 0, ops._ptr(y), cout, ops._ptr(ws), fws,
         ops._stream())
    torch.cuda.synchronize()
    lib.of_timing_enable(0)
    k_arr = (C.c_int * 8)()
    got = {k_arr[i] for i in range(lib.of_timing_read(8, k_arr, None, None))}
    assert 100 in got, got                      # conv_tile_bf16<128, 4, 2, 0, 8>
    xb = x.to(torch.bfloat16).double()
    wb = wt.to(torch.bfloat16).double()
    yref = R.conv2d_same(xb, wb, None, 1)
    assert rel_inf(y, yref) < 1e-5 and rel_l2(y, yref) < 1e-6


def test_conv_bf16_tall_dgrad():
    """bf16 input gradient on 8 x 32 output tiles (of_set_tuning key 18 = 1: grids of >= 1024
    tiles, BN 128) against the 4 x 32 tiles (key 18 = 0) and an fp64 transposed conv of the
    bf16-rounded operands, with the LeakyReLU derivative of the producer in the epilogue."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_LEAKY, call
    lib = _lib.lib()
    n, h, w, cin, cout = 8, 128, 256, 128, 128
    dy = rng_tensor((n, h, w, cout), 43)
    src = rng_tensor((n, h, w, cin), 44)
    wt = rng_tensor((3, 3, cin, cout), 45, scale=(2.0 / (9 * cin)) ** 0.5)
    layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=1, act=ACT_LEAKY, cin_p=cin,
                          precision="bf16")
    d = layer.desc(n, h, w)
    _, wd = layer.packed(d)
    dyd, srcd = dev(dy), dev(src)      # (held: a temporary's block is reused by the next one)
    outs, kinds = {}, {}
    try:
        for form in (1, 0):
            assert lib.of_set_tuning(18, form) == 0
            dent, dws = layer.dgrad_entry(d)
            ws = torch.empty(dws // 4 + 4, device="cuda")
            dx = torch.empty(n, h, w, cin, device="cuda")
            lib.of_timing_read(0, None, None, None)
            lib.of_timing_enable(1)
            call(dent, C.byref(d), ops._ptr(dyd), cout, ops._ptr(wd), ops._ptr(srcd), cin,
                 ACT_LEAKY, 0.3, ops._ptr(dx), cin, ops._ptr(ws), dws, ops._stream())
            torch.cuda.synchronize()
            lib.of_timing_enable(0)
            k_arr = (C.c_int * 8)()
            kinds[form] = {k_arr[i] for i in range(lib.of_timing_read(8, k_arr, None, None))}
            outs[form] = dx
    finally:
        lib.of_set_tuning(18, 0)
        lib.of_timing_enable(0)
    assert 108 in kinds[1] and 108 not in kinds[0], kinds   # conv_tile_bf16<128, 4, 2, 1, 8>
    assert rel_inf(outs[1], outs[0]) < 1e-6
    dyb = dy.to(torch.bfloat16).double()
    wb = wt.to(torch.bfloat16).double()
    dref = torch.nn.grad.conv2d_input((n, cin, h, w), wb.permute(3, 2, 0, 1),
                                      dyb.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    dref = dref * torch.where(src.double() > 0, 1.0, 0.3)
    assert rel_inf(outs[1], dref) < 1e-5 and rel_l2(outs[1], dref) < 1e-6


# ----------------------------------------------------------------------- cost volume ----
CORR_FORM_DEFAULT = 5      # of_set_tuning key 9: bit 0 corr_fwd_blk, bit 1 corr_bwd_blk, bit 2 fused bwd


class _corr_form:
    """Select the cost-volume kernel forms for a block, restoring the defaults: bits 0-2 are
    of_set_tuning key 9 (bit 2: corr_bwd_fused), bit 3 key 19 (the gather backward on 8 x 16
    tiles)."""

    def __init__(self, form):
        self.form = form

    def __enter__(self):
        from optical_flow_amd import _lib
        assert _lib.lib().of_set_tuning(9, self.form & 7) == 0
        assert _lib.lib().of_set_tuning(19, (self.form >> 3) & 1) == 0

    def __exit__(self, *exc):
        from optical_flow_amd import _lib
        _lib.lib().of_set_tuning(9, CORR_FORM_DEFAULT)
        _lib.lib().of_set_tuning(19, 0)


@pytest.mark.parametrize("form", [1, 3, 0, 9, 5, 4])
@pytest.mark.parametrize("shape", [(2, 12, 20, 64), (1, 24, 32, 256), (2, 9, 13, 6), (1, 19, 70, 32),
                                   (3, 40, 56, 64), (1, 17, 35, 100)])
def test_cost_volume(form, shape):
    """Cost volume and both input gradients against fp64 autograd, for the register-blocked
    forms (key 9 = 3: persistent grid, slab groups with partial sums on small grids) and the
    per-pixel forms (key 9 = 0); ragged tiles, channel counts that are not a slab multiple
    and not a multiple of 4 (scalar loads)."""
    ops = _ops()
    f1, f2 = rng_tensor(shape, 1), rng_tensor(shape, 2)
    a, b = f64(f1).requires_grad_(True), f64(f2).requires_grad_(True)
    cv = R.create_cost_volume(a, b, 3)
    g = rng_tensor(tuple(cv.shape), 3)
    (cv * f64(g)).sum().backward()
    ad, bd = dev(f1).requires_grad_(True), dev(f2).requires_grad_(True)
    with _corr_form(form):
        cvd = ops.cost_volume(ad, bd, 3)
        assert rel_inf(cvd, cv) < REL_TOL
        (cvd * dev(g)).sum().backward()
        torch.cuda.synchronize()
    assert rel_inf(ad.grad, a.grad) < REL_TOL
    assert rel_inf(bd.grad, b.grad) < REL_TOL


@pytest.mark.parametrize("n,h,w,c,cp,has_flow", [(2, 8, 12, 64, 116, True),
                                                  (1, 19, 70, 64, 120, True),
                                                  (2, 24, 32, 256, 308, False),
                                                  (1, 9, 35, 6, 60, True),
                                                  # h >= 96: the strip-sweep kernels
                                                  (1, 100, 40, 64, 116, True),
                                                  (2, 97, 33, 128, 180, True),
                                                  (1, 96, 20, 6, 60, False),
                                                  (1, 4, 8, 128, 180, True),
                                                  (1, 2, 4, 256, 308, False),
                                                  (8, 48, 64, 128, 180, True)])
@pytest.mark.parametrize("form", [1, 3, 0, 9, 5, 4])
def test_corr_concat(form, n, h, w, c, cp, has_flow):
    """The fused concat([f1, cost volume, flow]) kernel and its gradient, for both kernel
    forms (key 9): multi-tile and ragged shapes, 1 to 8 channel slabs (and slab groups with
    partial sums), with and without flow, float4 and scalar paths."""
    ops = _ops()
    f1, f2, fl = rng_tensor((n, h, w, c), 4), rng_tensor((n, h, w, c), 5), rng_tensor((n, h, w, 2), 6)
    a, b, fo = [f64(t).requires_grad_(True) for t in (f1, f2, fl)]
    parts = [a, R.create_cost_volume(a, b, 3)] + ([fo] if has_flow else [])
    xo = torch.cat(parts, -1)
    used = xo.shape[-1]
    g = rng_tensor(tuple(xo.shape), 7)
    (xo * f64(g)).sum().backward()
    ad, bd, fd = [dev(t).requires_grad_(True) for t in (f1, f2, fl)]
    with _corr_form(form):
        xd = ops.corr_concat(ad, bd, fd if has_flow else None, 3, cp)
        assert rel_inf(xd[..., :used], xo) < REL_TOL
        assert xd[..., used:].abs().max().item() == 0
        gd = torch.zeros((n, h, w, cp), device="cuda")
        gd[..., :used] = dev(g)
        gd[..., used:] = 1.0        # gradient on the padding must not leak anywhere
        (xd * gd).sum().backward()
        torch.cuda.synchronize()
    pairs = ((ad, a), (bd, b)) + (((fd, fo),) if has_flow else ())
    for d_, o_ in pairs:
        assert rel_inf(d_.grad, o_.grad) < REL_TOL


@pytest.mark.parametrize("n,h,w,c,cp,has_flow", [(2, 24, 32, 64, 116, True), (1, 40, 72, 64, 116, True),
                                                  (4, 48, 64, 128, 180, True), (2, 96, 64, 64, 113, False)])
def test_corr_concat_fwd16(n, h, w, c, cp, has_flow):
    """of_corr_concat_fwd16: the concat row written as a bf16 image (ld16 channels) equals the
    RNE of of_corr_concat_fwd's fp32 row, with zeros past the row."""
    ops = _ops()
    from optical_flow_amd import _lib
    lib = _lib.lib()
    if lib.of_corr_concat_fwd16_ok(n, h, w, c) != 1:
        pytest.skip("grid needs slab groups")
    f1, f2, fl = [dev(rng_tensor(s_, 40 + k)) for k, s_ in
                  enumerate([(n, h, w, c), (n, h, w, c), (n, h, w, 2)])]
    fu = fl if has_flow else None
    ld16 = (cp + 31) // 32 * 32
    x = torch.empty(n, h, w, cp, device="cuda")
    wsb = lib.of_corr_fwd_workspace(n, h, w, c, 3)
    ws = torch.empty(wsb // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    from optical_flow_amd._lib import call
    call("of_corr_concat_fwd", P(f1), P(f2), P(fu), n, h, w, c, 3, P(x), cp, P(ws), wsb, st)
    x16 = torch.full((n, h, w, ld16), 7.0, dtype=torch.bfloat16, device="cuda")
    call("of_corr_concat_fwd16", P(f1), P(f2), P(fu), n, h, w, c, 3, P(x16), ld16, st)
    torch.cuda.synchronize()
    assert torch.equal(x16[..., :cp], x.bfloat16()), "image != RNE of the fp32 row"
    assert (x16[..., cp:] == 0).all(), "channels past the row must be zero"


# ------------------------------------------------------------------------------ warp ----
@pytest.mark.parametrize("shape,flow_scale", [((2, 12, 20, 64), 3.0), ((2, 16, 16, 128), 1.5),
                                              ((1, 10, 14, 3), 4.0), ((2, 8, 24, 32), 20.0),
                                              ((1, 4, 8, 128), 0.5), ((1, 40, 70, 64), 1.0),
                                              ((2, 70, 40, 32), 6.0), ((2, 30, 50, 64), 40.0)])
def test_warp(shape, flow_scale):
    ops = _ops()
    n, h, w, c = shape
    f2 = rng_tensor(shape, 11)
    fl = rng_tensor((n, h, w, 2), 12, scale=flow_scale)
    a, fo = f64(f2).requires_grad_(True), f64(fl).requires_grad_(True)
    out = R.warp_features(fo, a)
    g = rng_tensor(tuple(out.shape), 13)
    (out * f64(g)).sum().backward()
    ad, fd = dev(f2).requires_grad_(True), dev(fl).requires_grad_(True)
    od = ops.warp(ad, fd)
    assert rel_inf(od, out) < REL_TOL
    (od * dev(g)).sum().backward()
    assert rel_inf(ad.grad, a.grad) < REL_TOL
    assert rel_inf(fd.grad, fo.grad) < REL_TOL


@pytest.mark.parametrize("form", [1, 0])
@pytest.mark.parametrize("shape,flow_scale,offset", [((2, 40, 56, 64), 0.3, 0.0),
                                                     ((2, 24, 40, 128), 0.8, 0.0),
                                                     ((1, 33, 45, 64), 0.3, 30.0),
                                                     ((1, 33, 45, 64), 0.3, -30.0),
                                                     ((2, 20, 28, 64), 5.0, 0.0)])
def test_warp_bwd_forms(form, shape, flow_scale, offset):
    """Feature-warp backward with the tile scatter aggregated in LDS (of_set_tuning key 7 = 1:
    sub-pixel flows, clipped tiles on a border strip, and spread flows that fall back to direct
    atomics) and with the border-corner cache only (key 7 = 0), against fp64 autograd."""
    from optical_flow_amd import _lib
    ops = _ops()
    n, h, w, c = shape
    f2 = rng_tensor(shape, 31)
    fl = rng_tensor((n, h, w, 2), 32, scale=flow_scale) + offset
    a, fo = f64(f2).requires_grad_(True), f64(fl).requires_grad_(True)
    out = R.warp_features(fo, a)
    g = rng_tensor(tuple(out.shape), 33)
    (out * f64(g)).sum().backward()
    lib = _lib.lib()
    try:
        assert lib.of_set_tuning(7, form) == 0
        ad, fd = dev(f2).requires_grad_(True), dev(fl).requires_grad_(True)
        od = ops.warp(ad, fd)
        (od * dev(g)).sum().backward()
        torch.cuda.synchronize()
    finally:
        lib.of_set_tuning(7, 1)
    assert rel_inf(ad.grad, a.grad) < REL_TOL
    assert rel_inf(fd.grad, fo.grad) < REL_TOL


def test_bilinear_interpolation_absolute():
    from optical_flow_amd.transformations import bilinear_interpolation
    n, h, w, c = 2, 9, 11, 8
    inp = rng_tensor((n, h, w, c), 21)
    pts = rng_tensor((n, h, w, 2), 22, lo=-3.0, hi=14.0)
    a, po = f64(inp).requires_grad_(True), f64(pts).requires_grad_(True)
    out = R.bilinear_interpolation(a, po)
    g = rng_tensor(tuple(out.shape), 23)
    (out * f64(g)).sum().backward()
    ad, pd = dev(inp).requires_grad_(True), dev(pts).requires_grad_(True)
    od = bilinear_interpolation(ad, pd)
    assert rel_inf(od, out) < REL_TOL
    (od * dev(g)).sum().backward()
    assert rel_inf(ad.grad, a.grad) < REL_TOL
    assert rel_inf(pd.grad, po.grad) < REL_TOL


@pytest.mark.parametrize("absolute", [False, True], ids=["grid", "absolute"])
@pytest.mark.parametrize("shape,flow_scale,offset", [((2, 40, 56, 64), 0.3, 0.0),
                                                     ((2, 24, 40, 128), 0.8, 0.0),
                                                     ((1, 33, 45, 64), 0.3, 30.0),
                                                     ((1, 20, 24, 64), 0.3, -30.0),
                                                     ((2, 20, 28, 64), 5.0, 0.0),
                                                     ((2, 10, 14, 3), 4.0, 0.0),
                                                     ((1, 17, 23, 32), 2.0, 0.0),
                                                     ((1, 9, 11, 6), 1.0, 0.0),
                                                     ((1, 40, 24, 64), 1.0, 0.0),
                                                     ((1, 31, 29, 16), 2.5, 0.0),
                                                     ((2, 20, 60, 64), 0.5, 0.0),
                                                     ((1, 60, 20, 128), 0.5, 0.0),
                                                     ((1, 18, 56, 6), 0.4, 0.0),
                                                     ((8, 96, 128, 64), 1.5, 0.0)])
def test_warp_bwd_deterministic(shape, flow_scale, offset, absolute):
    """The deterministic warp backward (of_warp_bwd_det, ops.deterministic()): against fp64
    autograd of the reference sampler (transformations.py:85-129) for sub-pixel, spread and
    border-clipped flows (20 x 24 at offset -30: every sample clamps onto one corner pixel, the
    longest possible run), any channel count, grid + flow and absolute points, the window
    gather's pile row / column workgroups (|w - h| > 16, P1's transposed grid clips every
    source beyond h onto the last row); BITWISE equal
    over repeated launches; the atomic default agrees up to its add order."""
    from optical_flow_amd.transformations import bilinear_interpolation
    ops = _ops()
    n, h, w, c = shape
    f2 = rng_tensor(shape, 41)
    fl = rng_tensor((n, h, w, 2), 42, scale=flow_scale) + offset
    if absolute:
        fl = fl + torch.stack(torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij"),
                              -1).float()
    fwd_ref = R.bilinear_interpolation if absolute else R.warp_features
    a, fo = f64(f2).requires_grad_(True), f64(fl).requires_grad_(True)
    out = fwd_ref(a, fo) if absolute else fwd_ref(fo, a)
    g = rng_tensor(tuple(out.shape), 43)
    (out * f64(g)).sum().backward()
    fwd = (lambda x, f: bilinear_interpolation(x, f)) if absolute else (lambda x, f: ops.warp(x, f))
    runs = []
    with ops.deterministic():
        for _ in range(3):
            ad, fd = dev(f2).requires_grad_(True), dev(fl).requires_grad_(True)
            (fwd(ad, fd) * dev(g)).sum().backward()
            torch.cuda.synchronize()
            runs.append((ad.grad.clone(), fd.grad.clone()))
    assert rel_inf(runs[0][0], a.grad) < REL_TOL
    assert rel_inf(runs[0][1], fo.grad) < REL_TOL
    for gi, gf in runs[1:]:
        assert torch.equal(gi, runs[0][0]) and torch.equal(gf, runs[0][1])
    with ops.deterministic(False):
        ad, fd = dev(f2).requires_grad_(True), dev(fl).requires_grad_(True)
        (fwd(ad, fd) * dev(g)).sum().backward()             # the atomic form
    assert rel_inf(ad.grad, runs[0][0]) < REL_TOL
    assert rel_inf(fd.grad, runs[0][1]) < REL_TOL


@pytest.mark.parametrize("shape,flow_scale,offset", [((2, 32, 32, 64), 0.2, 0.0),
                                                     ((1, 48, 48, 128), 0.25, 0.0),
                                                     ((2, 24, 24, 12), 0.2, 0.0),
                                                     ((1, 40, 40, 64), 0.2, 0.6),
                                                     ((2, 20, 60, 64), 0.2, 0.0),
                                                     ((1, 40, 40, 64), 0.1, -6.0),
                                                     ((2, 36, 44, 128), 0.2, 0.0)])
def test_warp_bwd_det_paths(shape, flow_scale, offset):
    """of_warp_bwd_det's three ways to d(features) on one input: window mode A (of_set_tuning
    key 28 = 8, the default for these flows), mode B (key 28 = 1: centred windows, border pixels
    on workgroups of their own) and the fixed-point path (key 28 = 0) -- each against fp64;
    A and B BITWISE equal off the border (the same ascending (source, corner) order; B splits a
    border pixel's sum over 16 partials); the fixed-point sums within 1e-5 of A; d(flow) bitwise
    equal across all three (the same fixed-order kernel arithmetic)."""
    ops = _ops()
    from optical_flow_amd import _lib
    lib = _lib.lib()
    n, h, w, c = shape
    f2 = rng_tensor(shape, 51)
    fl = rng_tensor((n, h, w, 2), 52, scale=flow_scale) + offset
    g = rng_tensor(shape, 53)
    a, fo = f64(f2).requires_grad_(True), f64(fl).requires_grad_(True)
    (R.warp_features(fo, a) * f64(g)).sum().backward()
    res = {}
    try:
        for key in (8, 1, 0):
            assert lib.of_set_tuning(28, key) == 0
            with ops.deterministic(True):
                ad, fd = dev(f2).requires_grad_(True), dev(fl).requires_grad_(True)
                (ops.warp(ad, fd) * dev(g)).sum().backward()
            torch.cuda.synchronize()
            res[key] = (ad.grad.clone(), fd.grad.clone())
            assert rel_inf(res[key][0], a.grad) < REL_TOL, key
            assert rel_inf(res[key][1], fo.grad) < REL_TOL, key
    finally:
        lib.of_set_tuning(28, 8)
    assert torch.equal(res[8][0][:, 1:-1, 1:-1], res[1][0][:, 1:-1, 1:-1])
    assert rel_inf(res[0][0], res[8][0]) < 1e-5
    assert torch.equal(res[8][1], res[1][1]) and torch.equal(res[8][1], res[0][1])


@pytest.mark.parametrize("shape,scale,offset,mode", [
    ((2, 40, 56, 64), 0.5, 0.0, "A"),          # small flows: R <= 8
    ((2, 48, 64, 128), 1.5, 21.0, "B"),        # large smooth flows: piles on the borders
    ((1, 64, 48, 64), 1.5, -13.0, "B"),
    ((1, 20, 24, 6), 0.5, -30.0, "B"),         # everything clamped onto one corner pixel
    ((1, 30, 40, 64), 6.0, 0.0, "fixed"),      # large rough flows: no window
    ((1, 30, 40, 64), 0.3, 12.0, "fixed"),     # large, rough at 0.3 px noise: no window
])
def test_warp_bwd_det_modes(shape, scale, offset, mode):
    """of_warp_bwd_det's paths, read back from its workspace header (of_warp_bwd_det_header):
    mode A (R <= key 28), mode B (smooth fields: centred windows, every entry found -- the
    count is 4 n h w) and the fixed-point path (rough fields: no window); each against fp64 autograd
    of warp_features (model.py:55-73), bitwise equal over repeated launches."""
    import ctypes as C
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import call
    lib = _lib.lib()
    n, h, w, c = shape
    f2 = rng_tensor(shape, 61)
    if mode == "B":     # a smooth field (mode B is tried for neighbour changes <= 0.5 px)
        ii, jj = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")
        fl = offset + scale * torch.stack([torch.sin(0.21 * ii + 0.13 * jj),
                                           torch.cos(0.17 * ii - 0.11 * jj)], -1)
        fl = fl.expand(n, h, w, 2).contiguous()
    else:
        fl = rng_tensor((n, h, w, 2), 62, scale=scale) + offset
    g = rng_tensor(shape, 63)
    a, fo = f64(f2).requires_grad_(True), f64(fl).requires_grad_(True)
    (R.warp_features(fo, a) * f64(g)).sum().backward()
    wsb = lib.of_warp_bwd_det_workspace(n, h, w, c)
    hoff = lib.of_warp_bwd_det_header(n, h, w, c)
    outs = []
    dg, df2, dfl_in = dev(g), dev(f2), dev(fl)            # (kept alive across the launch)
    for _ in range(2):
        ws = torch.full(((wsb + 3) // 4,), -7, dtype=torch.int32, device="cuda")
        dinp = torch.full(shape, float("nan"), device="cuda")
        dfl = torch.empty((n, h, w, 2), device="cuda")
        P = lambda t: C.c_void_p(t.data_ptr())
        call("of_warp_bwd_det", P(dg), P(df2), n, h, w, c, P(dfl_in), 0, P(dinp), P(dfl),
             None, 0, P(ws), wsb, None)
        torch.cuda.synchronize()
        hdr = ws[hoff // 4: hoff // 4 + 64 * 129].cpu()
        outs.append((dinp.clone(), dfl.clone(), hdr))
    hdr = outs[0][2]
    rr = max(int(hdr[64 * (33 + k)]) for k in range(32))
    found = int(sum(int(hdr[64 * (1 + k)]) for k in range(32)))
    if mode == "A":
        assert rr <= 8 and found == 0, (rr, found)
    elif mode == "B":
        assert rr > 8 and found == 4 * n * h * w, (rr, found)
    else:
        assert rr > 8 and found != 4 * n * h * w, (rr, found)
    assert rel_inf(outs[0][0], a.grad) < REL_TOL
    assert rel_inf(outs[0][1], fo.grad) < REL_TOL
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_warp_bwd_det_nonfinite_flow():
    """A NaN flow pixel: the float-atomic form writes NaN into the rows its clamped sample
    lands on; the deterministic form (no window covers a non-finite field: fixed point) must
    not return a finite d(features) either -- it writes NaN throughout -- and stays
    reproducible; d(flow) is NaN at that pixel in both."""
    ops = _ops()
    shape = (1, 20, 24, 16)
    n, h, w, c = shape
    f2 = dev(rng_tensor(shape, 71))
    fl = rng_tensor((n, h, w, 2), 72, scale=0.5)
    fl[0, 5, 7, 0] = float("nan")
    g = dev(rng_tensor(shape, 73))
    res = {}
    for det in (True, False):
        with ops.deterministic(det):
            ad, fd = f2.clone().requires_grad_(True), dev(fl).requires_grad_(True)
            (ops.warp(ad, fd) * g).sum().backward()
        torch.cuda.synchronize()
        res[det] = (ad.grad.clone(), fd.grad.clone())
    assert not torch.isfinite(res[False][0]).all()       # (the atomic form's NaN rows)
    assert not torch.isfinite(res[True][0]).all()
    assert torch.isnan(res[True][1][0, 5, 7]).any() and torch.isnan(res[False][1][0, 5, 7]).any()


@pytest.mark.parametrize("n,h,w,cin,cout,stride,prec,res", [
    (8, 96, 128, 64, 64, 1, "fp32", False),      # conv_tile_x3 one slice
    (8, 96, 128, 64, 64, 1, "fp32", True),       # + the BN layer's residual
    (16, 96, 128, 64, 128, 2, "fp32", True),     # conv_gemm_x3, stride-2 phase groups
    (8, 96, 128, 64, 64, 1, "bf16", True),       # conv_tile_bf16
])
def test_dgrad_bnp_partials(n, h, w, cin, cout, stride, prec, res):
    """of_conv2d_dgrad_add_act_bnp + of_bn_bwd_final: the input gradient t bitwise equal to
    of_conv2d_dgrad_add_act's, and the BN gradients of the layer whose output is act_src
    (inference BN, FusedBatchNormGrad: dbeta = sum t, dgamma = sum t zhat with zhat =
    (y - res - beta) / gamma, dbias = dgamma's scale s = gamma / sqrt(var + eps) times sum t)
    against a float64 reduction of that t, within 1e-5."""
    import ctypes as C
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_RELU, call
    lib = _lib.lib()
    wt = dev(rng_tensor((3, 3, cin, cout), 71, scale=(2.0 / (9 * cin)) ** 0.5))
    b = dev(rng_tensor((cout,), 72, scale=0.1))
    layer = ops.ConvLayer(wt, b, stride=stride, act=ACT_RELU, cin_p=cin, precision=prec)
    d = layer.desc(n, h, w)
    _, wd = layer.packed(d)
    dy = dev(rng_tensor((n, d.ho, d.wo, cout), 73))
    y = torch.relu(dev(rng_tensor((n, h, w, cin), 74)))            # the BN layer's output
    add = dev(rng_tensor((n, h, w, cin), 75))
    gamma = dev(rng_tensor((cin,), 76, scale=0.5)) + 1.0
    beta = dev(rng_tensor((cin,), 77, scale=0.2))
    var = dev(rng_tensor((cin,), 78, scale=0.1)).abs() + 0.5
    rres = dev(rng_tensor((n, h, w, cin), 79)) if res else None
    _, wsz = layer.dgrad_add_entry(d)
    ws = torch.empty(max(wsz, 4) // 4 + 4, device="cuda")
    P, st = ops._ptr, ops._stream()
    dx0 = torch.empty(n, h, w, cin, device="cuda")
    call("of_conv2d_dgrad_add_act", C.byref(d), layer.mode(d), P(dy), cout, P(wd), P(add), cin,
         P(y), cin, ACT_RELU, 0.0, P(dx0), cin, P(ws), wsz, st)
    pb = lib.of_conv2d_dgrad_bnp_bytes(C.byref(d))
    assert pb > 0
    part = torch.empty(pb // 4 + 4, device="cuda")
    nblk = C.c_int(0)
    dx = torch.empty_like(dx0)
    rc = lib.of_conv2d_dgrad_add_act_bnp(
        C.byref(d), layer.mode(d), P(dy), cout, P(wd), P(add), cin, P(y), cin, ACT_RELU,
        C.c_float(0.0), P(dx), cin, P(gamma), P(beta), P(rres), cin if res else 0, P(part), pb,
        C.byref(nblk), P(ws), wsz, st)
    assert rc == 0, lib.of_last_error()
    assert nblk.value > 0
    out = [torch.zeros(cin, device="cuda") for _ in range(3)]
    call("of_bn_bwd_final", P(part), nblk.value, cin, P(gamma), P(var), 1e-3, P(out[0]),
         P(out[1]), P(out[2]), 0, st)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx0)
    t = f64(dx).reshape(-1, cin)
    zhat = (f64(y) - (f64(rres) if res else 0.0) - f64(beta)).reshape(-1, cin) / f64(gamma)
    s = f64(gamma) / torch.sqrt(f64(var) + 1e-3)
    want = ((t * zhat).sum(0), t.sum(0), t.sum(0) * s)
    for name, got, ref in zip(("dgamma", "dbeta", "dbias"), out, want):
        e = rel_l2(got, ref)
        print("%s %s rel_l2 %.2e" % (prec, name, e))
        assert e < 1e-5, (name, e)
