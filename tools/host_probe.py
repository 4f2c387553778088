"""Host-side issue time of the eager train step vs its GPU time (is the step host-bound?).

python tools/host_probe.py   (GPU): 20 steps issued back to back; prints the host time to
issue them (no sync) and the wall time to finish, per step, plus a per-phase host breakdown
(forward / loss / backward / optimizer issue) of one synchronised step."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from optical_flow_amd import _lib  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.loss import LossLayer  # noqa: E402
from optical_flow_amd.model import FlowNet  # noqa: E402
from optical_flow_amd.params import flow_net_spec, init_params  # noqa: E402
from optical_flow_amd.train import KerasAdam, Trainer  # noqa: E402

_lib.load()
H, W, B = 384, 512, 8
net = FlowNet(H, W, values=init_params(flow_net_spec(), 0), precision="fp32")
tr = Trainer(net, KerasAdam(net.store), LossLayer())
batch = torch.from_numpy(synthetic_batch(B, H, W, seed=1234)).cuda()
for i in range(8):
    tr.train_step(batch, i)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for i in range(n):
    tr.train_step(batch, 8 + i)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("issue %.3f ms/step, finish %.3f ms/step" % ((t1 - t0) / n * 1e3, (t2 - t0) / n * 1e3))
# one step, phases timed on the host with a sync before it (host issue cost alone)
torch.cuda.synchronize()
ph = {}
t = time.perf_counter()
store = net.store
store.zero_grad()
flows = net(batch)
ph["forward"] = time.perf_counter() - t
t = time.perf_counter()
loss = tr.loss_layer(batch, flows)
ph["loss"] = time.perf_counter() - t
t = time.perf_counter()
loss.backward()
ph["backward"] = time.perf_counter() - t
t = time.perf_counter()
tr.optimizer.apply_gradients()
ph["optimizer"] = time.perf_counter() - t
torch.cuda.synchronize()
print("host issue per phase (ms):", {k: round(v * 1e3, 3) for k, v in ph.items()})
