"""Kernel-level parity for the small kernels of the step (restored after round 5 dropped them
from test_gpu_kernels.py): photometric L1 (the multi-level forward / backward
entry points through the C ABI, odd level sizes, padded d(flow) rows), flow upscale, max-pool,
Keras Adam, the stem's fused max-pool / BN / ReLU backward, split-K against unsplit convs and
the in-place input gradient with an added gradient.  Each against the CPU oracle (float64) or
torch autograd in float64 on the same seeded inputs; REL_TOL = 1e-3."""
import ctypes as C

import pytest
import torch

from helpers import REL_TOL, dev, f64, rel_inf, rel_l2, rng_tensor
from oracle import ref_flow as R

pytestmark = pytest.mark.gpu


def _ops():
    from optical_flow_amd import ops
    return ops


# ------------------------------------------------------------------- photometric loss ---
@pytest.mark.parametrize("size", [(2, 64, 96), (1, 128, 256), (1, 48, 80), (3, 80, 112)])
def test_photometric_loss(size):
    """LossLayer (loss.py:5-32) end to end through ops.photometric_loss: loss and every
    level's d(flow).  (1, 48, 80) and (3, 80, 112) give odd level sizes (3 x 5, 5 x 7 at
    H/16) and partial blocks everywhere."""
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.loss import LossLayer
    n, H, W = size
    batch = torch.from_numpy(synthetic_batch(n, H, W, seed=5))
    flows = [rng_tensor((n, H >> (s + 1), W >> (s + 1), 2), 50 + s, scale=2.0) for s in range(4)]
    fo = [f64(f).requires_grad_(True) for f in flows]
    lo = R.photometric_loss(f64(batch), fo)
    lo.backward()
    fd = [dev(f).requires_grad_(True) for f in flows]
    ld = LossLayer()(dev(batch), fd)
    assert abs(ld.item() - lo.item()) / abs(lo.item()) < REL_TOL
    ld.backward()
    for a, b in zip(fd, fo):
        assert rel_l2(a.grad, b.grad) < REL_TOL


@pytest.mark.parametrize("with_dloss", [True, False])
@pytest.mark.parametrize("levels", [[(5, 7), (13, 21), (1, 3), (40, 57)], [(96, 128)],
                                    [(2, 2), (33, 65)]])
def test_photo_l1_multi_kernels(levels, with_dloss):
    """of_photo_l1_fwd_multi / of_photo_l1_bwd_multi directly: per level l (any h x w, not a
    pyramid), the level's slice of the partials sums to sum |img1 - warp(img2, flow)|
    (loss.py:26-28), and d(flow) = coef_l * dloss * d/dflow of that sum, written at row
    stride 4 into a padded buffer whose padding stays untouched; dloss NULL means 1."""
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import call
    ops = _ops()
    n, L = 2, len(levels)
    imgs = [rng_tensor((n, h, w, 6), 200 + i) for i, (h, w) in enumerate(levels)]
    flows = [rng_tensor((n, h, w, 2), 300 + i, scale=3.0) for i, (h, w) in enumerate(levels)]
    coefs = [0.5 + 0.25 * i for i in range(L)]
    dl = 1.75 if with_dloss else 1.0
    di, dfl = [dev(t) for t in imgs], [dev(t) for t in flows]
    hs = (C.c_int * L)(*[h for h, _ in levels])
    ws = (C.c_int * L)(*[w for _, w in levels])
    nparts = [_lib.lib().of_photo_l1_partials(n, h, w) for h, w in levels]
    parts = torch.empty(sum(nparts), device="cuda")
    P = ops._ptr
    call("of_photo_l1_fwd_multi", (C.c_void_p * L)(*[t.data_ptr() for t in di]),
         (C.c_void_p * L)(*[t.data_ptr() for t in dfl]), n, hs, ws, L, P(parts), ops._stream())
    outs = [torch.full((n, h, w, 4), 7.0, device="cuda") for h, w in levels]
    dloss = torch.tensor([dl], device="cuda") if with_dloss else None
    call("of_photo_l1_bwd_multi", (C.c_void_p * L)(*[t.data_ptr() for t in di]),
         (C.c_void_p * L)(*[t.data_ptr() for t in dfl]), n, hs, ws, L,
         (C.c_float * L)(*coefs), P(dloss), (C.c_void_p * L)(*[o.data_ptr() for o in outs]),
         (C.c_int * L)(*([4] * L)), ops._stream())
    torch.cuda.synchronize()
    off = 0
    for i in range(L):
        img, fl = f64(imgs[i]), f64(flows[i]).requires_grad_(True)
        s = (img[..., :3] - R.warp_features(fl, img[..., 3:])).abs().sum()
        (s * coefs[i] * dl).backward()
        got = parts[off:off + nparts[i]].double().sum().item()
        off += nparts[i]
        assert abs(got - s.item()) / s.item() < REL_TOL, (i, got, s.item())
        assert rel_l2(outs[i][..., :2], fl.grad) < REL_TOL, i
        assert torch.equal(outs[i][..., 2:], torch.full_like(outs[i][..., 2:], 7.0))


# -------------------------------------------------------------------------- upscale -----
@pytest.mark.parametrize("shape", [(2, 6, 8, 2), (1, 24, 32, 2), (2, 5, 7, 3), (1, 2, 4, 2)])
def test_upscale(shape):
    """upscale_flow (model.py:76-77): resize x2 (half-pixel bilinear) times 2.0, and its
    adjoint."""
    ops = _ops()
    x = rng_tensor(shape, 31)
    xo = f64(x).requires_grad_(True)
    yo = R.upscale_flow(xo)
    g = rng_tensor(tuple(yo.shape), 32)
    (yo * f64(g)).sum().backward()
    xd = dev(x).requires_grad_(True)
    yd = ops.upscale2x(xd, 2.0)
    assert rel_inf(yd, yo) < REL_TOL
    (yd * dev(g)).sum().backward()
    assert rel_inf(xd.grad, xo.grad) < REL_TOL


# ------------------------------------------------------------------------- max pool -----
@pytest.mark.parametrize("shape", [(2, 8, 12, 64), (1, 10, 6, 4), (3, 14, 22, 128)])
def test_maxpool(shape):
    """MaxPool2D() (model.py:17): forward exact, gradient to the window's maximum."""
    ops = _ops()
    x = rng_tensor(shape, 41)
    xo = f64(x).requires_grad_(True)
    yo = R.maxpool2(xo)
    g = rng_tensor(tuple(yo.shape), 42)
    (yo * f64(g)).sum().backward()
    xd = dev(x).requires_grad_(True)
    yd = ops.maxpool2(xd)
    assert rel_inf(yd, yo) == 0.0
    (yd * dev(g)).sum().backward()
    assert rel_inf(xd.grad, xo.grad) < REL_TOL


# ------------------------------------------------------------------------------ adam ----
@pytest.mark.parametrize("gscale", [1.0, 0.125])
def test_keras_adam(gscale):
    """Keras Adam (train.py:34,56; P13, epsilon-hat form) over a parameter arena for three
    steps against the oracle's; gscale: the data-parallel 1/world folded into the launch."""
    from optical_flow_amd.model import ParamStore
    from optical_flow_amd.params import head_spec, init_params
    from optical_flow_amd.train import KerasAdam
    spec = head_spec(3)
    vals = init_params(spec, 3)
    store = ParamStore(spec, vals, device="cuda")
    opt = KerasAdam(store, learning_rate=1e-2)
    ref = R.KerasAdam(lr=1e-2)
    pref = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    for it in range(3):
        grads = {k: rng_tensor(v.shape, 100 + it * 7 + i) for i, (k, v) in enumerate(vals.items())}
        for k, g in grads.items():
            store.params[k]._of_grad.copy_(g.cuda())
        opt.apply_gradients(grad_scale=gscale)
        ref.step(pref, {k: g.double() * gscale for k, g in grads.items()})
    assert opt.iterations == 3
    for k in vals:
        assert rel_inf(store.params[k], pref[k]) < 1e-5, k


# ------------------------------------------------------- stem fused max-pool backward ---
@pytest.mark.parametrize("from_y", [False, True])
@pytest.mark.parametrize("n,h,w,c,with_g", [(2, 8, 12, 64, True), (1, 6, 10, 16, False),
                                            (3, 34, 70, 64, True),
                                            # many workgroups, a ragged last one; 8 quads
                                            (2, 96, 130, 64, True), (1, 40, 52, 32, False)])
def test_maxpool_bn_act_bwd_fused(n, h, w, c, with_g, from_y):
    """The stem's fused backward (max-pool backward + out0's second gradient + BN/ReLU
    backward, model.py:12-17) against torch autograd of relu(bn(z)) -> {out0, maxpool} in
    float64; from_y: of_maxpool_bn_relu_bwd, z not stored (zhat recovered from y)."""
    from optical_flow_amd._lib import call, lib
    torch.manual_seed(0)
    z = torch.randn(n, h, w, c, dtype=torch.float64)
    gamma = 1 + 0.2 * torch.rand(c, dtype=torch.float64)
    beta = 0.1 * torch.randn(c, dtype=torch.float64)
    mean = 0.1 * torch.randn(c, dtype=torch.float64)
    var = 1 + 0.2 * torch.rand(c, dtype=torch.float64)
    dyp = torch.randn(n, h // 2, w // 2, c, dtype=torch.float64)
    g = torch.randn(n, h, w, c, dtype=torch.float64) if with_g else None
    zr = z.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    y = torch.relu((zr - mean) * (gr / torch.sqrt(var + 1e-3)) + br)
    pooled = torch.nn.functional.max_pool2d(y.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    loss = (pooled * dyp).sum() + ((y * g).sum() if with_g else 0)
    loss.backward()
    yv = y.detach()

    def dv(t):
        return t.float().cuda().contiguous()

    outs = [torch.empty(n, h, w, c, device="cuda")] + [torch.zeros(c, device="cuda")
                                                       for _ in range(3)]
    ws = torch.empty(lib().of_maxpool_bn_act_bwd_workspace(n, h, w, c) // 4 + 1, device="cuda")

    def P(t):
        return C.c_void_p(t.data_ptr()) if t is not None else None

    args = [dv(dyp), dv(g) if with_g else None, dv(yv), dv(z), dv(gamma), dv(mean), dv(var)]
    if from_y:
        call("of_maxpool_bn_relu_bwd", n, h, w, c, P(args[0]), P(args[1]), P(args[2]),
             P(args[4]), P(dv(beta)), P(args[6]), 1e-3, P(outs[0]), P(outs[1]), P(outs[2]),
             P(outs[3]), 0, P(ws), None)
    else:
        call("of_maxpool_bn_act_bwd", n, h, w, c, *[P(t) for t in args], 1e-3, P(outs[0]),
             P(outs[1]), P(outs[2]), P(outs[3]), 0, P(ws), None)
    torch.cuda.synchronize()
    dz, dg, db, dbias = [o.double().cpu() for o in outs]
    exp_dbias = zr.grad.sum(dim=(0, 1, 2))
    for got, exp in [(dz, zr.grad), (dg, gr.grad), (db, br.grad), (dbias, exp_dbias)]:
        assert ((got - exp).abs().max() / exp.abs().max()).item() < 1e-5


# ------------------------------------------------------------- split-K vs unsplit conv ---
@pytest.mark.parametrize("stride", [1, 2])
def test_conv_split_k_matches_unsplit(stride):
    """Small grids split K over workgroups (fp32 slabs + epilogue pass); without workspace
    the same call runs unsplit.  Both must agree (and match the oracle)."""
    from optical_flow_amd._lib import ACT_LEAKY, call, lib
    ops = _ops()
    n, h, w, cin, cout, k = 2, 12, 16, 64, 128, 3
    x = dev(rng_tensor((n, h, w, cin), 71))
    wt = dev(rng_tensor((k, k, cin, cout), 72, scale=0.05))
    b = dev(rng_tensor((cout,), 73, scale=0.1))
    layer = ops.ConvLayer(wt, b, stride=stride, act=ACT_LEAKY, f32_split=False)
    d = layer.desc(n, h, w)
    wf, wd = layer.packed(d)
    fws = lib().of_conv2d_fwd_workspace(C.byref(d))
    dws = lib().of_conv2d_dgrad_workspace(C.byref(d))
    assert fws > 0 and dws > 0, "this shape must take the split-K path"
    ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
    P, s = ops._ptr, ops._stream()
    y1 = torch.empty(n, d.ho, d.wo, cout, device="cuda")
    y2 = torch.empty_like(y1)
    call("of_conv2d_fwd", C.byref(d), P(x), cin, P(wf), P(b), None, None, None, None, 1e-3, None,
         0, ACT_LEAKY, 0.3, None, 0, P(y1), cout, P(ws), fws, s)
    call("of_conv2d_fwd", C.byref(d), P(x), cin, P(wf), P(b), None, None, None, None, 1e-3, None,
         0, ACT_LEAKY, 0.3, None, 0, P(y2), cout, None, 0, s)
    yo = R.leaky_relu(R.conv2d_same(f64(x), f64(wt), f64(b), stride))
    assert rel_inf(y1, yo) < REL_TOL and rel_inf(y2, yo) < REL_TOL
    assert rel_inf(y1, y2) < 1e-5
    g = dev(rng_tensor(tuple(y1.shape), 74))
    dx1 = torch.empty_like(x)
    dx2 = torch.empty_like(x)
    call("of_conv2d_dgrad", C.byref(d), P(g), cout, P(wd), P(x), cin, ACT_LEAKY, 0.3, P(dx1), cin,
         P(ws), dws, s)
    call("of_conv2d_dgrad", C.byref(d), P(g), cout, P(wd), P(x), cin, ACT_LEAKY, 0.3, P(dx2), cin,
         None, 0, s)
    xo = f64(x).requires_grad_(True)
    (R.conv2d_same(xo, f64(wt), None, stride) * f64(g)).sum().backward()
    ref = torch.where(f64(x) > 0, xo.grad, 0.3 * xo.grad)
    assert rel_inf(dx1, ref) < REL_TOL and rel_inf(dx2, ref) < REL_TOL


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("k,s", [(1, 2), (3, 2), (3, 1)])
def test_dgrad_add_in_place(k, s, prec):
    """The input gradient with an added gradient (dgrad_add entry of the layer's precision)
    with dx == add (in-place accumulation; 1x1 stride 2 then launches only the phase group a
    tap reaches) equals the out-of-place result bitwise."""
    from optical_flow_amd._lib import ACT_NONE, call
    ops = _ops()
    n, h, w, cin, cout = 2, 16, 20, 64, 128
    wt = dev(rng_tensor((k, k, cin, cout), 7, scale=0.1))
    layer = ops.ConvLayer(wt, dev(rng_tensor((cout,), 8)), stride=s, act=ACT_NONE, cin_p=cin,
                          precision=prec)
    d = layer.desc(n, h, w)
    _, wd = layer.packed(d)
    dy = dev(rng_tensor((n, d.ho, d.wo, cout), 9))
    add = dev(rng_tensor((n, h, w, cin), 10))
    entry, wsz = layer.dgrad_add_entry(d)
    P = ops._ptr
    ws = torch.empty(wsz // 4 + 1, device="cuda")
    out = torch.empty_like(add)
    call(entry, C.byref(d), P(dy), cout, P(wd), P(add), cin, P(out), cin, P(ws), wsz, None)
    inplace = add.clone()
    call(entry, C.byref(d), P(dy), cout, P(wd), P(inplace), cin, P(inplace), cin, P(ws), wsz,
         None)
    torch.cuda.synchronize()
    assert torch.equal(inplace, out)
    xo = torch.zeros(n, h, w, cin, dtype=torch.float64, requires_grad=True)
    (R.conv2d_same(xo, f64(wt), None, s) * f64(dy)).sum().backward()
    tol = REL_TOL if prec == "fp32" else 2e-2
    assert rel_l2(out - add, xo.grad) < tol


# ------------------------------------------ deterministic warp backward: tiled mode A ---
DET_TPRE_DEFAULT = 0          # of_set_tuning key 35's default (warp_det.hip g_det_tpre)

@pytest.mark.parametrize("shape,flow_scale,offset,rmax", [
    ((2, 40, 56, 64), 0.3, 0.0, 8),       # sub-pixel flows, pile row (w - h > 16)
    ((2, 24, 40, 128), 0.8, 0.0, 8),      # two channel blocks
    ((1, 33, 45, 64), 0.3, 3.0, 8),       # ragged tiles, samples piled towards an edge
    ((1, 20, 24, 64), 0.3, -3.0, 8),      # samples clamped onto the first row / column
    ((2, 20, 28, 64), 2.0, 0.0, 8),       # R = 8: the widest window
    ((2, 10, 14, 3), 1.0, 0.0, 8),        # scalar path (c % 4 != 0), tiny image
    ((1, 17, 23, 32), 1.0, 0.0, 8),
    ((1, 40, 24, 64), 0.5, 0.0, 8),       # pile column (h - w > 16)
    ((1, 31, 29, 16), 1.5, 0.0, 8),       # last row / column take the scan
    ((1, 30, 30, 64), 0.05, 0.0, 8),      # converging samples: bins beyond TILE_CAP
    ((1, 36, 36, 64), 6.0, 0.0, 16),      # large R (key 28 = 16)
    ((8, 96, 128, 64), 0.3, 0.0, 8)])     # a bench level
def test_warp_bwd_det_tiled_bitwise(shape, flow_scale, offset, rmax):
    """Mode A of of_warp_bwd_det by destination tiles (of_set_tuning key 34 = 1: inside
    own_window; 2, the default: own_tile, a kernel of its own) against the per-destination scan (key 34 =
    0): d(features) and d(flow) BITWISE equal
    (every destination sums its (source, corner) hits in ascending code order either way),
    and against fp64 autograd of warp_features (model.py:55-73)."""
    from optical_flow_amd import _lib
    ops = _ops()
    lib = _lib.lib()
    n, h, w, c = shape
    f2 = rng_tensor(shape, 81)
    fl = rng_tensor((n, h, w, 2), 82, scale=flow_scale) + offset
    if flow_scale == 0.05:     # every source of a 6 x 6 block sampling one point: deep bins
        fl = torch.zeros((n, h, w, 2))
        ii, jj = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")
        fl[0, ..., 0] = (torch.div(jj, 6, rounding_mode="floor") * 6 + 2.5) - ii
        fl[0, ..., 1] = (torch.div(ii, 6, rounding_mode="floor") * 6 + 2.5) - jj
        fl = fl * 0.25 + rng_tensor((n, h, w, 2), 83, scale=0.05)
    g = rng_tensor(shape, 84)
    a, fo = f64(f2).requires_grad_(True), f64(fl).requires_grad_(True)
    (R.warp_features(fo, a) * f64(g)).sum().backward()
    res = {}
    try:
        assert lib.of_set_tuning(28, rmax) == 0
        for tiled, pre in ((1, 0), (1, 1), (2, 0), (0, 0)):
            assert lib.of_set_tuning(34, tiled) == 0 and lib.of_set_tuning(35, pre) == 0
            with ops.deterministic(True):
                ad, fd = dev(f2).requires_grad_(True), dev(fl).requires_grad_(True)
                (ops.warp(ad, fd) * dev(g)).sum().backward()
            torch.cuda.synchronize()
            res[tiled, pre] = (ad.grad.clone(), fd.grad.clone())
    finally:
        lib.of_set_tuning(34, 2)
        lib.of_set_tuning(35, DET_TPRE_DEFAULT)
        lib.of_set_tuning(28, 8)
    assert rel_inf(res[1, 0][0], a.grad) < REL_TOL
    assert rel_inf(res[1, 0][1], fo.grad) < REL_TOL
    for k in ((1, 0), (1, 1), (2, 0)):   # (key 35: d(flow)'s loads issued first; key 34 = 2:
        # the tiles in own_tile, the last row / column and overflowed bins in own_window)
        assert torch.equal(res[k][0], res[0, 0][0]), (k, rel_inf(res[k][0], res[0, 0][0]))
        assert torch.equal(res[k][1], res[0, 0][1]), k


# ------------------------------------------------------- fp32 split 64-column tile forms ---
@pytest.mark.parametrize("n,h,w,cin,cout", [(8, 192, 256, 96, 64),    # level-1 c3: tall grid
                                            (8, 192, 256, 64, 32),    # level-1 c4: dgrad N = 64
                                            (2, 37, 45, 64, 64),      # odd, partial tiles
                                            (4, 24, 32, 128, 64)])    # small grid, split K
def test_conv_x3_bn64_forms(n, h, w, cin, cout):
    """The 64-column forms of conv_tile_x3 (of_set_tuning key 36: 1 = the 4-wave 8 x 32 form on
    large grids, 2 = <64, 4, 1, MODE, 4, 1>, 3 = <64, 2, 2, MODE, 4, 1>) against the default
    <64, 4, 2, MODE, 4>, forward and input gradient: every output element accumulates the same
    products in the same order (chunk, tap, six split products), so unsplit grids are equal bit
    for bit; where the K-split plan changes with the slot count, within 2e-6 relative.  The
    timing kinds say the form ran (128 + 8 mode + 7)."""
    ops = _ops()
    from optical_flow_amd import _lib
    from optical_flow_amd._lib import ACT_NONE, call
    lib = _lib.lib()
    x = rng_tensor((n, h, w, cin), 121)
    wt = rng_tensor((3, 3, cin, cout), 122, scale=(2.0 / (9 * cin)) ** 0.5)
    layer = ops.ConvLayer(dev(wt), dev(torch.zeros(cout)), stride=1, act=ACT_NONE, cin_p=cin,
                          f32_split=True)
    d = layer.desc(n, h, w)
    dy = rng_tensor((n, d.ho, d.wo, cout), 123)
    wf, wd = layer.packed(d)
    P, st = ops._ptr, ops._stream()
    xd, dyd = dev(x), dev(dy)
    res = {}
    try:
        for key in (0, 1, 2, 3):
            assert lib.of_set_tuning(36, key) == 0
            fent, fws = layer.fwd_entry(d)
            dent, dws = layer.dgrad_entry(d)
            ws = torch.empty(max(fws, dws) // 4 + 4, device="cuda")
            y = torch.full((n, d.ho, d.wo, cout), float("nan"), device="cuda")
            dx = torch.full((n, h, w, cin), float("nan"), device="cuda")
            lib.of_timing_enable(1)
            call(fent, C.byref(d), P(xd), cin, P(wf), P(layer.bias), None, None, None, None,
                 1e-3, None, 0, ACT_NONE, 0.0, None, 0, P(y), cout, P(ws), fws, st)
            call(dent, C.byref(d), P(dyd), cout, P(wd), None, 0, ACT_NONE, 0.0, P(dx), cin,
                 P(ws), dws, st)
            torch.cuda.synchronize()
            kk = (C.c_int * 64)()
            cnt = lib.of_timing_read(64, kk, None, None)
            lib.of_timing_enable(0)
            res[key] = (y, dx, {kk[i] for i in range(cnt)})
    finally:
        lib.of_set_tuning(36, 0)
        lib.of_timing_enable(0)
    want = set()
    if cout == 64:
        want.add(128 + 7)
    if cin == 64:
        want.add(128 + 8 + 7)
    tall_ok = n * -(-h // 8) * -(-w // 32) >= 4 * 256
    for key in (1, 2, 3):
        y, dx, kinds = res[key]
        if key > 1 or tall_ok:
            assert want <= kinds, (key, want, kinds)
        assert torch.isfinite(y).all() and torch.isfinite(dx).all()
        for got, ref in ((y, res[0][0]), (dx, res[0][1])):
            if tall_ok:
                assert torch.equal(got, ref), (key, rel_inf(got, ref))
            else:
                assert rel_inf(got, ref) < 2e-6, (key, rel_inf(got, ref))


# ------------------------------------------------------------------- weight packing -----
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_pack_many_matches_per_layer(precision):
    """of_conv_pack_many -- every conv of the net in one launch, the bf16 / split forward images
    by 32 x 64 LDS tiles (round 6) -- against the per-layer packers (of_conv_pack_weights_bn /
    _x3 / _bf16 / fp32), bit for bit, forward and input-gradient images, the BN scale folded."""
    from optical_flow_amd._lib import call
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import flow_net_spec, init_params, perturb_params
    ops = _ops()
    P = ops._ptr
    net = FlowNet(64, 128, values=perturb_params(init_params(flow_net_spec(), 0), 3),
                  precision=precision)
    layers = net.conv_layers()
    packer = ops.ConvPacker(layers, lambda: 0)
    packer.ensure()
    torch.cuda.synchronize()
    modes = set()
    for L in layers:
        d = L.desc(1, 16, 16)
        m = L.mode(d)
        modes.add(m)
        wf, wd = L._wf.clone(), L._wd.clone()
        f2, b2 = torch.full_like(wf, float("nan")), torch.full_like(wd, float("nan"))
        if L.bn is not None and not L.bn_train:
            call("of_conv_pack_weights_bn", C.byref(d), m, P(L.kernel), P(f2), P(b2), P(L.bn[0]),
                 P(L.bn[3]), ops.BN_EPS, ops._stream())
        else:
            call(("of_conv_pack_weights", "of_conv_pack_weights_bf16", "of_conv_pack_weights_x3")[m],
                 C.byref(d), P(L.kernel), P(f2), P(b2), ops._stream())
        torch.cuda.synchronize()
        assert torch.equal(wf, f2), (L.name, "forward image")
        assert torch.equal(wd, b2), (L.name, "input-gradient image")
    assert (2 if precision == "fp32" else 1) in modes, modes
