"""Parity at the benchmarked sizes: the HIP train step against the CPU oracle at the
configurations bench.py measures, not only at the small test sizes.

  * config 2 (BASELINE.json configs[1]): 384x512, B=8, fp32 -- the headline bench line;
  * the reference's own training shape, 192x640, B=4 (train.py:15-21);
  * config 5: 768x1024, bf16, B=1 per GPU (the bf16 MFMA kernels against the oracle with the
    same bf16 operand rounding, oracle/ref_flow.py set_conv_precision).

One forward + photometric loss + backward (train.py:50-55; Adam is covered by
test_gpu_model.py::test_train_steps_trajectory) on identical weights and image pairs.  Bar
(BASELINE.json north star, tests/helpers.py REL_TOL): flows and loss within 1e-3 relative,
every one of the 108 trainable-weight gradients within 1e-3 relative L2; EPE printed.  The kernel forms
the planner picks depend on the grid size (8x32 output tiles, the 9-tap weight gradient, K
splits), so the config-2 case also asserts, through the timing kinds of of_timing_read, that
the forms the bench reports are the ones that ran here.

The oracle runs in float64 on the host cores (about 50 s for config 2 on 8 cores).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from helpers import REL_TOL, dev, rel_inf, rel_l2
from oracle import ref_flow as R

pytestmark = pytest.mark.gpu

# timing kinds (bench.py kind_parts) of the forms the config-2 bench line reports
# (BENCH_r02.json roofline.per_kernel): fwd / dgrad on 8 x 32 tiles of conv_tile_x3<128, 4, 2,
# 8> (128, 136), the 9-tap weight gradient conv_wgrad_tile_x3b<2, 4, 8, 1> (148), the stem
# conv_stem_x3 (184) and its weight gradient conv_wgrad_stem_x3 (185), the split implicit GEMMs
# of the stride-2 / 1x1 layers (160 + mode * 8 + cfg) and the narrow flow convs (7, 15, 23).
CFG2_KINDS = {128, 136, 148, 184, 7, 15, 23, 185}
GEMM_X3_FWD, GEMM_X3_DGRAD, GEMM_X3_WGRAD = range(160, 168), range(168, 176), range(176, 184)


def _run(H, W, B, precision="fp32", seed=0):
    from optical_flow_amd import _lib, ops
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params, perturb_params
    vals = perturb_params(init_params(flow_net_spec(), seed), seed + 1)
    batch = synthetic_batch(B, H, W, seed=1234 + seed)
    net = FlowNet(H, W, values=vals, precision=precision)
    lib = _lib.lib()
    bd = dev(torch.from_numpy(batch))
    net.store.zero_grad()
    lib.of_timing_read(0, None, None, None)
    ops.TIMING_TAGS = []
    lib.of_timing_enable(1)
    try:
        flows = net(bd)
        loss = LossLayer()(bd, flows)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        lib.of_timing_enable(0)
        tags, ops.TIMING_TAGS = ops.TIMING_TAGS, None
    cap = 4096
    kk, ff, mm = (C.c_int * cap)(), (C.c_double * cap)(), (C.c_float * cap)()
    n = lib.of_timing_read(cap, kk, ff, mm)
    kinds = [kk[i] for i in range(n)]
    assert len(tags) == n
    flows = [f.detach().cpu().double() for f in flows]
    grads = {k: g.detach().cpu().double() for k, g in net.store.grads().items()}
    hip = (float(loss), flows, grads)
    # split-K: the layers whose fwd / dgrad plan at these sizes needs slab workspace
    split = set()
    for L in net.conv_layers():
        for d in L._descs.values():
            if L.fwd_entry(d)[1] > 0:
                split.add((L.name, 0))
            if L.cout > 4 and L.name != "conv1" and L.dgrad_entry(d)[1] > 0:   # images: no dgrad
                split.add((L.name, 1))
    del net, flows, loss, bd
    torch.cuda.empty_cache()
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    R.set_conv_precision(precision)
    try:
        lo, fo, go = R.train_step(torch.tensor(batch, dtype=torch.float64), p,
                                  list(encoder_blocks()), None)
    finally:
        R.set_conv_precision("fp32")
    return hip, (float(lo), fo, go), list(zip(tags, kinds)), split, batch


def _epe(a, b):
    return (a - b).norm(dim=-1).mean().item()


def _residual_flips(batch, flows_hip, flows_ref):
    """Pixels whose photometric residual sign (loss.py:28) differs between the two flow sets,
    per scale: where a gradient disagreement would come from (a kink of |.|)."""
    out = []
    x = torch.tensor(batch, dtype=torch.float64)
    H, W = x.shape[1], x.shape[2]
    for s, (fh, fr) in enumerate(zip(flows_hip, flows_ref)):
        h, w = H >> (s + 1), W >> (s + 1)
        r = R.resize_bilinear(x, h, w)
        dh = r[..., :3] - R.warp_features(fh, r[..., 3:])
        dr = r[..., :3] - R.warp_features(fr, r[..., 3:])
        flips = (torch.sign(dh) != torch.sign(dr)).nonzero().tolist()
        out.append(flips[:8] + (["... %d total" % len(flips)] if len(flips) > 8 else []))
    return out


def _check(hip, ref, batch, grad_tol=REL_TOL, flow_tol=REL_TOL, label=""):
    loss_h, flows_h, grads_h = hip
    loss_r, flows_r, grads_r = ref
    for k in range(len(flows_h)):
        assert flows_h[k].shape == flows_r[k].shape
        print("%s flow%d rel_inf %.2e EPE %.3e px" % (label, 3 - k, rel_inf(flows_h[k], flows_r[k]),
                                                      _epe(flows_h[k], flows_r[k])))
    lrel = abs(loss_h - loss_r) / abs(loss_r)
    print("%s loss hip %.8e oracle %.8e rel %.2e" % (label, loss_h, loss_r, lrel))
    errs = sorted(((rel_l2(g, grads_r[n]), n) for n, g in grads_h.items()), reverse=True)
    print("%s %d gradients: worst rel_l2 %.2e (%s), median %.2e" % (
        label, len(errs), errs[0][0], errs[0][1], errs[len(errs) // 2][0]))
    bad_flow = [k for k in range(len(flows_h)) if not rel_inf(flows_h[k], flows_r[k]) < flow_tol]
    bad_grad = [(e, n) for e, n in errs if not e < grad_tol]
    if bad_grad or bad_flow:
        print("residual sign flips per scale:", _residual_flips(batch, flows_h, flows_r))
    assert not bad_flow, bad_flow
    assert lrel < REL_TOL, lrel
    assert all(torch.isfinite(g).all() for g in grads_h.values())
    return errs, bad_grad


def test_config2_384x512_b8_fp32():
    """The headline configuration, the kernel forms the bench runs included."""
    hip, ref, launches, split, batch = _run(384, 512, 8)
    errs, bad = _check(hip, ref, batch, label="cfg2")
    assert len(errs) == 108      # every trainable weight: 54 kernels / biases / BN gamma, beta
    assert not bad, bad[:5]
    kinds = {k for _, k in launches}
    assert CFG2_KINDS <= kinds, (CFG2_KINDS - kinds, sorted(kinds))
    for fam in (GEMM_X3_FWD, GEMM_X3_DGRAD, GEMM_X3_WGRAD):
        assert kinds & set(fam), sorted(kinds)
    # at least one layer runs a K-split plan here (enc.l4 / the coarse heads), and it ran
    ran = {t for t, _ in launches}
    assert split and split <= ran, (sorted(split), len(ran))
    print("cfg2: %d conv launches, %d kinds, K-split launches: %s" % (
        len(launches), len(kinds), sorted(split)))


def test_reference_shape_192x640_b4_fp32():
    """train.py:15-21: the shape the reference trains at (KITTI crops 192 x 640, batch 4)."""
    hip, ref, launches, split, batch = _run(192, 640, 4, seed=2)
    errs, bad = _check(hip, ref, batch, label="192x640")
    assert not bad, bad[:5]
    print("192x640: kinds %s, K-split layers %d" % (sorted({k for _, k in launches}), len(split)))


# bf16 end to end (see test_gpu_model.py BF16_*): flows 3e-2 relative, loss 1e-3, gradient
# relative L2 median < 8e-2 and worst < 0.25 -- the bench's bf16 bounds.
BF16_FLOW_TOL, BF16_GRAD_MEDIAN, BF16_GRAD_WORST = 3e-2, 8e-2, 2.5e-1


def test_config5_768x1024_bf16():
    """Config 5 per GPU (768 x 1024, bf16 MFMA convs, fp32 accumulation / master weights)
    against the oracle with the same bf16 operand rounding; B=1 keeps the float64 oracle in
    budget (the bench runs B=8 per GPU, same kernels and plans up to the batch dimension)."""
    hip, ref, launches, split, batch = _run(768, 1024, 1, precision="bf16", seed=4)
    errs, _ = _check(hip, ref, batch, grad_tol=BF16_GRAD_WORST, flow_tol=BF16_FLOW_TOL,
                     label="cfg5 bf16")
    assert errs[len(errs) // 2][0] < BF16_GRAD_MEDIAN, errs[len(errs) // 2]
    assert errs[0][0] < BF16_GRAD_WORST, errs[0]
    kinds = {k for _, k in launches}
    assert any(96 <= k < 128 for k in kinds), sorted(kinds)      # bf16 halo-tiled kernels ran


def test_config3_384x512_b32_bf16():
    """Config 3 (384 x 512, B = 32, bf16) at its own size: the kernel forms the B = 32 plans
    pick (the bf16-image flow heads at levels 2-3, conv_halo_b16 / conv_wgrad_b16i) checked
    against the bf16-rounded oracle on 2 of the 32 pairs -- the forward is per pair, and so is
    every gradient when the output gradient is zero on the other 30 pairs:
      * the whole net's forward: flows of pairs 3 and 17 (oracle on those 2 pairs);
      * the level-3 flow module (model.py:80-116; 54.7 % of the FLOPs) teacher-forced with the
        HIP encoder's features at B = 32 and an output gradient that is nonzero on pairs 3
        and 17 only: outputs, input gradients and all 12 weight / bias gradients against the
        oracle on those 2 pairs (the LeakyReLU slopes the HIP head took given to the oracle,
        as test_gpu_bf16_modules.py), 1e-2 relative L2."""
    from optical_flow_amd import _lib, ops
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params, perturb_params
    H, W, B, pick = 384, 512, 32, [3, 17]
    vals = perturb_params(init_params(flow_net_spec(), 11), 12)
    batch = synthetic_batch(B, H, W, seed=4321)
    net = FlowNet(H, W, values=vals, precision="bf16")
    lib = _lib.lib()
    bd = dev(torch.from_numpy(batch))
    lib.of_timing_read(0, None, None, None)
    lib.of_timing_enable(1)
    try:
        with torch.no_grad():
            flows = net(bd)
            torch.cuda.synchronize()
    finally:
        lib.of_timing_enable(0)
    cap = 4096
    kk, ff, mm = (C.c_int * cap)(), (C.c_double * cap)(), (C.c_float * cap)()
    kinds = {kk[i] for i in range(lib.of_timing_read(cap, kk, ff, mm))}
    assert {288, 289, 290, 291} <= kinds, sorted(kinds)     # bf16-image forward, BN 128..32
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    R.set_conv_precision("bf16")
    try:
        with torch.no_grad():
            fo = R.flow_net(torch.tensor(batch[pick], dtype=torch.float64), p,
                            list(encoder_blocks()))
    finally:
        R.set_conv_precision("fp32")
    for k in range(4):
        fh = flows[k][pick].double().cpu()
        e = rel_inf(fh, fo[k])
        print("cfg3 flow%d (pairs %s) rel_inf %.2e EPE %.3e px" % (3 - k, pick, e, _epe(fh, fo[k])))
        assert e < BF16_FLOW_TOL, (k, e)
    # ---- level-3 module, teacher-forced at B = 32, gradient on 2 pairs
    with torch.no_grad():
        feats = net.encoder.forward4(ops.split_pair(bd))
        f1, f2 = feats[0][:B].contiguous(), feats[0][B:].contiguous()
        prev = flows[1].contiguous()                        # level 2's flow (H/4)
    g = torch.zeros(B, H // 2, W // 2, 2, dtype=torch.float64)
    g[pick] = torch.tensor(np.random.default_rng(5).standard_normal((2, H // 2, W // 2, 2)))
    ins = [f1, f2, prev]
    hin = [t.detach().clone().requires_grad_(True) for t in ins]
    net.store.zero_grad()
    lib.of_timing_read(0, None, None, None)
    lib.of_timing_enable(1)
    try:
        out = net.heads[3](hin[0], hin[1], hin[2])
        acts = out.grad_fn.saved_tensors
        assert acts[1].dtype == torch.bfloat16               # the bf16-image path ran
        masks = [(a[pick] > 0).cpu() for a in acts[1:6]]
        (out * dev(g.float())).sum().backward()
        torch.cuda.synchronize()
    finally:
        lib.of_timing_enable(0)
    n = lib.of_timing_read(cap, kk, ff, mm)
    kinds = {kk[i] for i in range(n)}
    assert {296, 304} <= kinds, sorted(kinds)                # image dgrad + weight gradient
    prefix = "flow_module_3"
    names = ["%s/conv%d/%s" % (prefix, i, k) for i in range(6) for k in ("kernel", "bias")]
    grads = net.store.grads()
    leaves = [t[pick].detach().cpu().double().requires_grad_(True) for t in ins]
    ws = {nme: p[nme].clone().requires_grad_(True) for nme in names}
    pp = dict(p)
    pp.update(ws)
    R.set_conv_precision("bf16")
    try:
        o = R.flow_module(leaves[0], leaves[1], leaves[2], 3, pp, prefix, masks=masks)
        (o * g[pick]).sum().backward()
    finally:
        R.set_conv_precision("fp32")
    errs = [("out", rel_l2(out[pick], o.detach()))]
    errs += [("d_in%d" % i, rel_l2(h.grad[pick], l.grad)) for i, (h, l) in enumerate(zip(hin, leaves))]
    errs += [(nme, rel_l2(grads[nme], ws[nme].grad)) for nme in names]
    for e in errs:
        print("cfg3 level-3 module %-32s rel_l2 %.2e" % e)
    bad = [e for e in errs if not e[1] < 1e-2]
    assert not bad, bad
