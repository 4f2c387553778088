"""Per-tensor breakdown of the smoke() comparison (GPU): prints every gradient's rel-L2 error."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import ref_flow as R  # noqa: E402
from optical_flow_amd import _lib  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.loss import LossLayer  # noqa: E402
from optical_flow_amd.model import FlowNet  # noqa: E402
from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params, perturb_params  # noqa: E402

H, W, B, SEED, TOP = [int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (64, 128, 1, 42, 25))]
_lib.load()
vals = perturb_params(init_params(flow_net_spec(), 0), 1)
batch = synthetic_batch(B, H, W, seed=SEED)
net = FlowNet(H, W, values=vals)
bd = torch.from_numpy(batch).cuda()
net.store.zero_grad()
flows = net(bd)
loss = LossLayer()(bd, flows)
loss.backward()
torch.cuda.synchronize()
p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
lo, fo, go = R.train_step(torch.tensor(batch, dtype=torch.float64), p, list(encoder_blocks()), None)
print("== H W B seed", H, W, B, SEED, "loss", loss.item(), lo.item())
for i in range(4):
    a, b = flows[i].detach().double().cpu(), fo[i]
    print("flow", i, ((a - b).abs().max() / b.abs().max()).item())
errs = []
for n, g in net.store.grads().items():
    a, b = g.detach().double().cpu(), go[n]
    errs.append((((a - b).norm() / b.norm().clamp_min(1e-30)).item(), n, tuple(a.shape),
                 b.norm().item()))
for e in sorted(errs, reverse=True)[:TOP]:
    print("%.3e %-40s %s |ref| %.3e" % e)
