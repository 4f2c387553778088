"""Flow magnitudes reaching the feature warp in the bench step (synthetic batch, init weights)."""
import sys, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from optical_flow_amd import ops, _lib
from optical_flow_amd.data import synthetic_batch
from optical_flow_amd.loss import LossLayer
from optical_flow_amd.model import FlowNet
from optical_flow_amd.params import flow_net_spec, init_params
from optical_flow_amd.train import KerasAdam, Trainer
_lib.load()
H, W, B = 384, 512, 8
net = FlowNet(H, W, values=init_params(flow_net_spec(), 0), precision="fp32")
tr = Trainer(net, KerasAdam(net.store), LossLayer())
batch = torch.from_numpy(synthetic_batch(B, H, W, seed=1234)).cuda()
orig = ops.warp
log = []
def warp(inp, flow):
    a = flow.detach().abs().amax(-1).flatten().float()
    q = torch.quantile(a[torch.randperm(a.numel(), device=a.device)[:100000]], torch.tensor([0.5, 0.99, 0.999], device=a.device))
    log.append((tuple(flow.shape), float(a.max()), [round(float(v), 3) for v in q], float((a > 6).float().mean())))
    return orig(inp, flow)
ops.warp = warp
for step in range(12):
    log.clear()
    tr.train_step(batch, step)
    torch.cuda.synchronize()
    if step in (0, 1, 5, 11):
        print("step", step)
        for l in log: print("  ", l)
