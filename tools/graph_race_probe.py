"""Which gradients does a captured train step compute in a different order than the eager one?

Run with DEBUG_HIP_FORCE_GRAPH_QUEUES=1: HIP then executes a captured graph on the launch
stream alone, in a topological order of the graph's edges -- so two kernels on different
streams that the capture left unordered run in an order unrelated to the eager step's timing.
With the deterministic warp backward a replay must equal the eager step bitwise; a gradient
that differs (by rounding: two accumulations into one buffer in the other order) names a
missing cross-stream edge.  Prints per parameter the max |diff| and its rel l2.

    DEBUG_HIP_FORCE_GRAPH_QUEUES=1 python tools/graph_race_probe.py [fp32|bf16] [inference|training]

(Round 6: the graph is captured on one stream by default, ops.single_stream; PROBE_CLEAR_POOL=1
empties FlowGrad's buffer pool after the capture, so the eager trainer does not share the
captured graph's pooled buffers.)
"""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch  # noqa: E402

from optical_flow_amd import ops  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.model import FlowNet  # noqa: E402
from optical_flow_amd.params import flow_net_spec, init_params, perturb_params  # noqa: E402
from optical_flow_amd.train import KerasAdam, Trainer  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
bn_mode = sys.argv[2] if len(sys.argv) > 2 else "inference"
H, W, B = 128, 256, 2
vals = perturb_params(init_params(flow_net_spec(), 3), 4)


def trainer():
    net = FlowNet(H, W, values=vals, precision=prec, bn_mode=bn_mode)
    return Trainer(net, KerasAdam(net.store, learning_rate=1e-4))


def sync(dst, src):
    dst.flow_net.store.arena.copy_(src.flow_net.store.arena)
    dst.flow_net.store.buffers.copy_(src.flow_net.store.buffers)
    dst.flow_net.store.version += 1
    for name in ("m", "v", "_iter", "_sched"):
        getattr(dst.optimizer, name).copy_(getattr(src.optimizer, name))


batches = [torch.from_numpy(synthetic_batch(B, H, W, seed=40 + i)).cuda() for i in range(3)]
with ops.deterministic(True):
    gt, eager = trainer(), trainer()
    step = gt.graphed(batches[0].clone(), warmup=1)
    if os.environ.get("PROBE_CLEAR_POOL") == "1":   # the eager trainer gets buffers of its own
        ops.FlowGrad._pool.clear()
    for k in (1, 2):
        sync(eager, gt)
        le, _ = eager.train_step(batches[k])
        lg, _ = step(batches[k])
        torch.cuda.synchronize()
        ge, gg = eager.flow_net.store.grads(), gt.flow_net.store.grads()
        bad = []
        for n in ge:
            d = (gg[n] - ge[n]).abs().max().item()
            if d > 0:
                rel = ((gg[n] - ge[n]).norm() / ge[n].norm().clamp_min(1e-30)).item()
                bad.append((rel, d, n))
        bad.sort(reverse=True)
        print("%s %s replay %d: loss %r vs %r; %d of %d gradients differ" % (
            prec, bn_mode, k, float(lg), float(le), len(bad), len(ge)), flush=True)
        for rel, d, n in bad[:40]:
            print("   %-42s rel_l2 %.2e  max|diff| %.2e" % (n, rel, d), flush=True)
print("queues:", os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES"))
