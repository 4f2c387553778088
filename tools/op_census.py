"""Which torch ops run inside one training step (copies, fills, cats that are not ours)?
python tools/op_census.py   (GPU) -- prints aten ops by count for one step with their callers."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from optical_flow_amd import _lib
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import flow_net_spec, init_params
    from optical_flow_amd.train import KerasAdam, Trainer
    _lib.load()
    net = FlowNet(384, 512, values=init_params(flow_net_spec(), 0))
    trainer = Trainer(net, KerasAdam(net.store), LossLayer())
    batch = torch.from_numpy(synthetic_batch(8, 384, 512, seed=1234)).cuda()
    for i in range(3):
        trainer.train_step(batch, i)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        trainer.train_step(batch, 3)
        torch.cuda.synchronize()
    cnt = Counter()
    where = {}
    for ev in prof.events():
        if ev.name.startswith("aten::") and ev.name not in ("aten::empty", "aten::empty_like",
                                                              "aten::empty_strided", "aten::view",
                                                              "aten::as_strided", "aten::detach",
                                                              "aten::slice", "aten::select",
                                                              "aten::permute", "aten::reshape",
                                                              "aten::alias", "aten::_unsafe_view",
                                                              "aten::unsqueeze", "aten::t",
                                                              "aten::resolve_conj", "aten::resolve_neg",
                                                              "aten::lift_fresh", "aten::record_stream",
                                                              "aten::result_type", "aten::expand"):
            cnt[ev.name] += 1
            st = [f for f in (ev.stack or []) if "optical_flow_amd" in f or "bench" in f]
            where.setdefault(ev.name, Counter())[" <- ".join(st[:3])] += 1
    for name, c in cnt.most_common(40):
        print("%5d %s" % (c, name))
        for w, k in where[name].most_common(4):
            print("        %3d  %s" % (k, w[:200]))


if __name__ == "__main__":
    main()
