"""Uninitialised-read probe: every torch.empty of the step is filled with NaN
(torch.use_deterministic_algorithms + torch.utils.deterministic.fill_uninitialized_memory), so a
kernel that reads memory nothing in the step wrote turns its outputs NaN (or different).  One
eager train step against the same step without the fill (same state, deterministic warp
backward): prints the gradients that are non-finite or differ.
python tools/uninit_probe.py [fp32|bf16] [inference|training] [H W B]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from optical_flow_amd import ops  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.model import FlowNet  # noqa: E402
from optical_flow_amd.params import flow_net_spec, init_params, perturb_params  # noqa: E402
from optical_flow_amd.train import KerasAdam, Trainer  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
bn_mode = sys.argv[2] if len(sys.argv) > 2 else "inference"
H, W, B = [int(v) for v in sys.argv[3:6]] if len(sys.argv) > 5 else (128, 256, 2)
vals = perturb_params(init_params(flow_net_spec(), 3), 4)
batch = torch.from_numpy(synthetic_batch(B, H, W, seed=41)).cuda()


def step(fill):
    torch.use_deterministic_algorithms(fill, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = fill
    net = FlowNet(H, W, values=vals, precision=prec, bn_mode=bn_mode)
    tr = Trainer(net, KerasAdam(net.store, learning_rate=1e-4))
    loss, flows = tr.train_step(batch)
    torch.cuda.synchronize()
    out = ({n: g.clone() for n, g in net.store.grads().items()}, float(loss),
           [f.clone() for f in flows])
    torch.use_deterministic_algorithms(False)
    return out


with ops.deterministic(True):
    ref, lref, fref = step(False)
    for rep in range(2):
        got, lgot, fgot = step(True)
        bad = []
        for n in ref:
            fin = bool(torch.isfinite(got[n]).all())
            if not fin or not torch.equal(got[n], ref[n]):
                e = ((got[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-30)).item()
                bad.append((n, fin, e))
        fl = [bool(torch.equal(a, b)) for a, b in zip(fgot, fref)]
        print("%s %s %dx%d B=%d NaN-filled empties, run %d: loss %r vs %r, flows equal %s, "
              "%d gradients non-finite or different" % (prec, bn_mode, H, W, B, rep, lgot, lref,
                                                         fl, len(bad)), flush=True)
        for n, fin, e in bad[:40]:
            print("   %-42s finite %s rel_l2 %.2e" % (n, fin, e), flush=True)
