"""Regenerate the golden fixtures from the CPU oracle (float64).  Run from the repo root:
    python tests/golden/make_golden.py
Inputs are regenerated from seeds (data.synthetic_batch, params.init_params), so the fixtures
only hold outputs: flows, loss, and gradients (full for the small head, summaries for the
full model).  The oracle restates the reference semantics; TF itself is absent (parity
unpinned), so these fixtures pin the oracle and the HIP path to each other across rounds."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import ref_flow as R  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.params import (encoder_blocks, flow_net_spec, init_params,  # noqa: E402
                                     perturb_params, two_layer_head_spec)

OUT = os.path.dirname(os.path.abspath(__file__))


def head_case():
    """Config 1: 2-layer head, 128x256 pairs, batch 2 (BASELINE.json configs[0])."""
    vals = perturb_params(init_params(two_layer_head_spec(), 7), 8)
    batch = synthetic_batch(2, 128, 256, seed=11)
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    loss, flows, grads = R.train_step(torch.tensor(batch, dtype=torch.float64), p, None, None,
                                      model="head")
    out = {"loss": np.array(loss.item()), "flow0": flows[0].numpy().astype(np.float32)}
    for k, g in grads.items():
        out["grad:" + k] = g.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "head2_128x256_b2.npz"), **out)


def full_case():
    """Full flow net at 64x128, batch 1, perturbed seed-0 weights."""
    vals = perturb_params(init_params(flow_net_spec(), 0), 1)
    batch = synthetic_batch(1, 64, 128, seed=21)
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    loss, flows, grads = R.train_step(torch.tensor(batch, dtype=torch.float64), p,
                                      list(encoder_blocks()), None)
    out = {"loss": np.array(loss.item())}
    for i, f in enumerate(flows):
        out["flow%d" % i] = f.numpy().astype(np.float32)
    names = sorted(grads)
    out["grad_names"] = np.array(names)
    out["grad_l2"] = np.array([grads[k].norm().item() for k in names])
    out["grad_sum"] = np.array([grads[k].sum().item() for k in names])
    out["grad_head16"] = np.stack([np.pad(grads[k].flatten()[:16].numpy(),
                                          (0, max(0, 16 - grads[k].numel())))
                                   for k in names]).astype(np.float64)
    np.savez_compressed(os.path.join(OUT, "flownet_64x128_b1.npz"), **out)


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    head_case()
    full_case()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
