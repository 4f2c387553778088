"""End-to-end parity of the HIP flow net against the CPU oracle (float64) on identical
weights and image pairs: the 4 flow fields, the loss, every trainable-weight gradient, and a
short Keras-Adam trajectory.  Tolerance 1e-3 relative (BASELINE.json north star); EPE between
the HIP flows and the oracle flows is reported."""
import numpy as np
import pytest
import torch

from helpers import REL_TOL, dev, rel_inf, rel_l2
from oracle import ref_flow as R

pytestmark = pytest.mark.gpu


def _setup(H, W, B, seed=0):
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params, perturb_params
    vals = perturb_params(init_params(flow_net_spec(), seed), seed + 1)
    net = FlowNet(H, W, values=vals)
    batch = synthetic_batch(B, H, W, seed=1234 + seed)
    return net, vals, batch, list(encoder_blocks())


def epe(a, b):
    d = (a.detach().double().cpu() - b.detach().double().cpu())
    return d.norm(dim=-1).mean().item()


@pytest.mark.parametrize("H,W,B", [(64, 128, 2), (128, 256, 1)])
def test_flow_net_forward_backward(H, W, B):
    from optical_flow_amd.loss import LossLayer
    net, vals, batch, blocks = _setup(H, W, B)
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    loss_o, flows_o, grads_o = R.train_step(torch.tensor(batch, dtype=torch.float64), p, blocks,
                                            None)
    net.store.zero_grad()
    bd = dev(torch.from_numpy(batch))
    flows = net(bd)
    loss = LossLayer()(bd, flows)
    loss.backward()
    torch.cuda.synchronize()
    for k in range(4):
        assert flows[k].shape == flows_o[k].shape
        e = rel_inf(flows[k], flows_o[k])
        print("flow%d rel_inf %.2e EPE %.3e" % (3 - k, e, epe(flows[k], flows_o[k])))
        assert e < REL_TOL
    assert abs(loss.item() - loss_o.item()) / abs(loss_o.item()) < REL_TOL
    worst = 0.0
    for name, g in net.store.grads().items():
        e = rel_l2(g, grads_o[name])
        worst = max(worst, e)
        assert e < REL_TOL, "grad %s rel_l2 %.3e" % (name, e)
    print("worst grad rel_l2 %.2e" % worst)


def test_train_steps_trajectory():
    from optical_flow_amd.train import KerasAdam, Trainer
    net, vals, batch, blocks = _setup(64, 128, 2, seed=3)
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    opt_o = R.KerasAdam(lr=1e-4)
    trainer = Trainer(net, KerasAdam(net.store, learning_rate=1e-4))
    bd = dev(torch.from_numpy(batch))
    bo = torch.tensor(batch, dtype=torch.float64)
    for step in range(5):
        lo, _, _ = R.train_step(bo, p, blocks, opt_o)
        ld, _ = trainer.train_step(bd, step)
        rel = abs(ld.item() - lo.item()) / abs(lo.item())
        print("step %d loss hip %.6e oracle %.6e rel %.2e" % (step, ld.item(), lo.item(), rel))
        assert rel < REL_TOL
    for name in net.weight_names:
        assert rel_l2(net.store.params[name], p[name]) < REL_TOL, name
