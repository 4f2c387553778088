"""bf16 (configs 3-5) module by module, teacher-forced: every flow_module (model.py:80-116) and
every encoder stage (model.py:10-26: the stem and each residual block) gets the oracle's own
bf16-path inputs, rounded to fp32, and a fixed random output gradient; its output, input
gradients and weight gradients are compared with the oracle run in float64 with the same bf16
operand rounding (oracle/ref_flow.py set_conv_precision("bf16")).

End to end the bf16 comparison has to be statistical (test_gpu_model.py::test_flow_net_bf16):
the loss's |.| and the sampler's floor() turn 1e-3 flow differences into flipped gradient
contributions.  Feeding each module identical inputs and a smooth objective (sum(out * G))
removes that amplification, so a module whose bf16 kernels are wrong by more than bf16
rounding fails here at 1e-2 relative L2, whichever module it is.  Inside a flow module the
five LeakyReLUs are kinks of the same kind (a pre-activation within bf16 rounding of 0 takes
slope 1 on one side and 0.3 on the other); the flow-module cases therefore give the oracle the
slopes the HIP head took (oracle/ref_flow.py flow_head masks=) and print the comparison
against the oracle's own slopes beside it.
"""
import numpy as np
import pytest
import torch

from helpers import dev, rel_l2
from oracle import ref_flow as R

pytestmark = pytest.mark.gpu

TOL = 1e-2
H, W, B = 128, 256, 2


@pytest.fixture(scope="module")
def setup():
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params, perturb_params
    vals = perturb_params(init_params(flow_net_spec(), 6), 7)
    batch = synthetic_batch(B, H, W, seed=99)
    net = FlowNet(H, W, values=vals, precision="bf16")
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    blocks = list(encoder_blocks())
    x = torch.tensor(batch, dtype=torch.float64)
    imgs = torch.cat([x[..., :3], x[..., 3:]], 0)            # the Siamese (2B) batch
    R.set_conv_precision("bf16")
    try:
        with torch.no_grad():
            # the oracle's encoder, recording every stage input
            stage_in = [imgs]
            y = torch.relu(R.batchnorm_inference(
                R.conv2d_same(imgs, p["ResNet18/conv1/kernel"], p["ResNet18/conv1/bias"], 2),
                p, "ResNet18/layer1_bn"))
            feats = [y]
            y = R.maxpool2(y)
            for i, (prefix, cin, cout, stride, proj) in enumerate(blocks):
                stage_in.append(y)
                y = R.resnet_block(y, p, prefix, stride, proj)
                if i % 2 == 1:
                    feats.append(y)
            flows = R.flow_net(x, p, blocks)[::-1]            # coarse -> fine
    finally:
        R.set_conv_precision("fp32")
    return net, p, blocks, stage_in, feats, flows


def _oracle_grads(fn, inputs, p, names, g):
    """fn(*inputs) in float64 with bf16 operand rounding; returns (out, input grads, weight
    grads) of sum(out * g)."""
    leaves = [t.detach().clone().requires_grad_(True) for t in inputs]
    ws = [p[n].detach().clone().requires_grad_(True) for n in names]
    pp = dict(p)
    pp.update(zip(names, ws))
    R.set_conv_precision("bf16")
    try:
        out = fn(*leaves, pp)
        (out * g).sum().backward()
    finally:
        R.set_conv_precision("fp32")
    return out.detach(), [t.grad for t in leaves], {n: w.grad for n, w in zip(names, ws)}


def _compare(label, out_h, dins_h, grads_h, ref):
    out_r, dins_r, grads_r = ref
    errs = [("out", rel_l2(out_h, out_r))]
    errs += [("d_in%d" % i, rel_l2(a, b)) for i, (a, b) in enumerate(zip(dins_h, dins_r))
             if b is not None]
    errs += [(n, rel_l2(grads_h[n], grads_r[n])) for n in grads_r]
    worst = max(errs, key=lambda e: e[1])
    print("%-28s worst %-40s %.2e  (out %.2e)" % (label, worst[0], worst[1], errs[0][1]))
    bad = [e for e in errs if not e[1] < TOL]
    assert not bad, (label, bad)


def _rand_like(t, seed):
    r = np.random.default_rng(seed)
    return torch.tensor(r.standard_normal(tuple(t.shape)), dtype=torch.float64)


@pytest.mark.parametrize("img16", [False, True], ids=["f32img", "bf16img"])
@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_flow_module_bf16_teacher_forced(setup, level, img16, monkeypatch):
    """img16: the head runs on bf16 activation images and the conv_halo_b16 / conv_wgrad_b16i
    kernels (ops._img16_ok, forced here for every level by B16I_MIN_TILES = 0); otherwise
    (threshold above the grid) on the fp32-activation halo kernels."""
    from optical_flow_amd import ops
    monkeypatch.setattr(ops, "B16I_MIN_TILES", 0 if img16 else 1 << 30)
    net, p, blocks, stage_in, feats, flows = setup
    f = feats[3 - level]
    n = f.shape[0] // 2
    f1, f2 = f[:n].float().double(), f[n:].float().double()
    prev = flows[level - 1].float().double() if level > 0 else None
    prefix = "flow_module_%d" % level
    names = ["%s/conv%d/%s" % (prefix, i, k) for i in range(6) for k in ("kernel", "bias")]
    g = _rand_like(flows[level], 100 + level)
    ins = [f1, f2] + ([prev] if prev is not None else [])
    hin = [dev(t.float()).requires_grad_(True) for t in ins]
    net.store.zero_grad()
    out = net.heads[level](hin[0], hin[1], hin[2] if prev is not None else None)
    # the slopes the HIP head took: its saved LeakyReLU outputs (the conv stack's autograd
    # node keeps them for the fused activation-derivative epilogues)
    acts = out.grad_fn.saved_tensors
    assert (acts[1].dtype == torch.bfloat16) == img16          # the path the test asked for
    masks = [(a > 0).cpu() for a in acts[1:6]]
    (out * dev(g.float())).sum().backward()
    torch.cuda.synchronize()
    grads = net.store.grads()
    hip = (out, [t.grad for t in hin], {k: grads[k] for k in names})

    def fm(mk):
        return lambda a, b, *rest: R.flow_module(a, b, rest[0] if len(rest) == 2 else None, 3,
                                                 rest[-1], prefix, masks=mk)
    # for the record: against the oracle's own slopes, pre-activations within bf16 rounding of
    # 0 flip LeakyReLU'(z) between 1 and 0.3 (measured 1-2.4 % relative L2 on some gradients)
    free = _oracle_grads(fm(None), ins, p, names, g)
    worst_free = max(rel_l2(hip[2][n], free[2][n]) for n in names)
    print("%s against the oracle's own LeakyReLU slopes: worst weight grad %.2e" % (prefix,
                                                                                     worst_free))
    ref = _oracle_grads(fm(masks), ins, p, names, g)
    _compare(prefix, *hip, ref)


def _stage_names(prefix, proj):
    convs = ["conv_a", "conv_b"] + (["proj"] if proj else [])
    bns = ["bn_a", "bn_b"] + (["bn_proj"] if proj else [])
    return (["%s/%s/%s" % (prefix, c, k) for c in convs for k in ("kernel", "bias")] +
            ["%s/%s/%s" % (prefix, b, k) for b in bns for k in ("gamma", "beta")])


@pytest.mark.parametrize("i", list(range(6)))
def test_res_block_bf16_teacher_forced(setup, i):
    from optical_flow_amd import ops
    net, p, blocks, stage_in, feats, flows = setup
    prefix, cin, cout, stride, proj = blocks[i]
    x = stage_in[i + 1].float().double()
    names = _stage_names(prefix, proj)
    with torch.no_grad():
        R.set_conv_precision("bf16")
        try:
            shape = R.resnet_block(x, p, prefix, stride, proj).shape
        finally:
            R.set_conv_precision("fp32")
    g = _rand_like(torch.empty(shape), 200 + i)
    ref = _oracle_grads(lambda a, pp: R.resnet_block(a, pp, prefix, stride, proj), [x], p, names, g)
    a, b, pj = net.encoder.blocks[i]
    xh = dev(x.float()).requires_grad_(True)
    net.store.zero_grad()
    out = ops.res_block(xh, a, b, pj)
    (out * dev(g.float())).sum().backward()
    torch.cuda.synchronize()
    grads = net.store.grads()
    _compare(prefix, out, [xh.grad], {k: grads[k] for k in names}, ref)


def test_stem_bf16_teacher_forced(setup):
    """conv1 7x7/2 + BN + ReLU (model.py:12-15) on the (2B) image batch: output and weight /
    BN gradients (the images take no gradient)."""
    net, p, blocks, stage_in, feats, flows = setup
    imgs = stage_in[0].float().double()
    names = ["ResNet18/conv1/kernel", "ResNet18/conv1/bias", "ResNet18/layer1_bn/gamma",
             "ResNet18/layer1_bn/beta"]

    def stem(a, pp):
        return torch.relu(R.batchnorm_inference(
            R.conv2d_same(a, pp["ResNet18/conv1/kernel"], pp["ResNet18/conv1/bias"], 2),
            pp, "ResNet18/layer1_bn"))

    g = _rand_like(feats[0], 300)
    ref = _oracle_grads(stem, [imgs], p, names, g)
    ref = (ref[0], [None], ref[2])
    x4 = torch.cat([dev(imgs.float()), torch.zeros(imgs.shape[:3] + (1,), device="cuda")], -1)
    net.store.zero_grad()
    out = net.encoder.conv1(x4)
    (out * dev(g.float())).sum().backward()
    torch.cuda.synchronize()
    grads = net.store.grads()
    _compare("stem", out, [None], {k: grads[k] for k in names}, ref)
