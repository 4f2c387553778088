"""Eager train steps with the side streams (default) against eager steps with every kernel on
the current stream (ops.single_stream), from the same state each step, deterministic warp
backward: every gradient must agree bitwise.  A difference that appears only from the second
step on points at state carried between steps.  python tools/eager_order_probe.py [steps]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from optical_flow_amd import ops  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.model import FlowNet  # noqa: E402
from optical_flow_amd.params import flow_net_spec, init_params, perturb_params  # noqa: E402
from optical_flow_amd.train import KerasAdam, Trainer  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
H, W, B = 128, 256, 2
vals = perturb_params(init_params(flow_net_spec(), 3), 4)


def trainer():
    net = FlowNet(H, W, values=vals)
    return Trainer(net, KerasAdam(net.store, learning_rate=1e-4))


def sync(dst, src):
    dst.flow_net.store.arena.copy_(src.flow_net.store.arena)
    dst.flow_net.store.version += 1
    for name in ("m", "v", "_iter", "_sched"):
        getattr(dst.optimizer, name).copy_(getattr(src.optimizer, name))


batches = [torch.from_numpy(synthetic_batch(B, H, W, seed=40 + i)).cuda() for i in range(steps)]
with ops.deterministic(True):
    a, b = trainer(), trainer()
    for k in range(steps):
        sync(b, a)
        la, _ = a.train_step(batches[k])
        with ops.single_stream():
            lb, _ = b.train_step(batches[k])
        torch.cuda.synchronize()
        ga, gb = a.flow_net.store.grads(), b.flow_net.store.grads()
        bad = sorted((((gb[n] - ga[n]).norm() / ga[n].norm().clamp_min(1e-30)).item(), n)
                     for n in ga if not torch.equal(ga[n], gb[n]))[::-1]
        print("step %d: loss %r vs %r, %d of %d gradients differ %s" % (
            k, float(la), float(lb), len(bad), len(ga),
            " ".join("%s:%.1e" % (n, e) for e, n in bad[:6])), flush=True)
