"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the oracle):
CPU -- the oracle still reproduces them; GPU -- the HIP path matches them (1e-3 relative)."""
import os

import numpy as np
import pytest
import torch

from helpers import REL_TOL, dev, rel_inf, rel_l2
from oracle import ref_flow as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with np.load(os.path.join(GOLD, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _head_inputs():
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.params import init_params, perturb_params, two_layer_head_spec
    vals = perturb_params(init_params(two_layer_head_spec(), 7), 8)
    return vals, synthetic_batch(2, 128, 256, seed=11)


def _full_inputs():
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.params import flow_net_spec, init_params, perturb_params
    vals = perturb_params(init_params(flow_net_spec(), 0), 1)
    return vals, synthetic_batch(1, 64, 128, seed=21)


def test_oracle_reproduces_head_fixture():
    g = _load("head2_128x256_b2.npz")
    vals, batch = _head_inputs()
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    loss, flows, grads = R.train_step(torch.tensor(batch, dtype=torch.float64), p, None, None,
                                      model="head")
    assert abs(loss.item() - float(g["loss"])) <= 1e-7 * abs(float(g["loss"]))
    np.testing.assert_allclose(flows[0].numpy(), g["flow0"], rtol=1e-5, atol=1e-6)
    for k, v in grads.items():
        np.testing.assert_allclose(v.numpy(), g["grad:" + k], rtol=1e-4, atol=1e-7)


def test_oracle_reproduces_full_fixture():
    from optical_flow_amd.params import encoder_blocks
    g = _load("flownet_64x128_b1.npz")
    vals, batch = _full_inputs()
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    loss, flows, grads = R.train_step(torch.tensor(batch, dtype=torch.float64), p,
                                      list(encoder_blocks()), None)
    assert abs(loss.item() - float(g["loss"])) <= 1e-7 * abs(float(g["loss"]))
    for i, f in enumerate(flows):
        np.testing.assert_allclose(f.numpy(), g["flow%d" % i], rtol=1e-4, atol=1e-6)
    names = list(g["grad_names"])
    l2 = np.array([grads[k].norm().item() for k in names])
    np.testing.assert_allclose(l2, g["grad_l2"], rtol=1e-6)


@pytest.mark.gpu
def test_hip_head_matches_fixture():
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import TwoLayerHead
    g = _load("head2_128x256_b2.npz")
    vals, batch = _head_inputs()
    net = TwoLayerHead(128, 256, values=vals)
    net.store.zero_grad()
    bd = dev(torch.from_numpy(batch))
    flows = net(bd)
    loss = LossLayer()(bd, flows)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(g["loss"])) / abs(float(g["loss"])) < REL_TOL
    assert rel_inf(flows[0], torch.tensor(g["flow0"])) < REL_TOL
    for k, v in net.store.grads().items():
        assert rel_l2(v, torch.tensor(g["grad:" + k])) < REL_TOL, k


@pytest.mark.gpu
def test_hip_flownet_matches_fixture():
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import FlowNet
    g = _load("flownet_64x128_b1.npz")
    vals, batch = _full_inputs()
    net = FlowNet(64, 128, values=vals)
    net.store.zero_grad()
    bd = dev(torch.from_numpy(batch))
    flows = net(bd)
    loss = LossLayer()(bd, flows)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(g["loss"])) / abs(float(g["loss"])) < REL_TOL
    for i in range(4):
        assert rel_inf(flows[i], torch.tensor(g["flow%d" % i])) < REL_TOL
    grads = net.store.grads()
    names = list(g["grad_names"])
    l2 = np.array([grads[k].norm().item() for k in names])
    np.testing.assert_allclose(l2, g["grad_l2"], rtol=REL_TOL)
    h16 = np.stack([np.pad(grads[k].flatten()[:16].cpu().numpy(),
                           (0, max(0, 16 - grads[k].numel()))) for k in names])
    scale = np.abs(g["grad_head16"]).max(axis=1, keepdims=True) + 1e-30
    assert (np.abs(h16 - g["grad_head16"]) / scale).max() < REL_TOL
