"""Host enqueue cost of one training step vs its GPU time (is the step launch-bound?).

python tools/host_time.py [--steps 10] [--graph]   (GPU)
enqueue ms = host time for train_step() to return (no sync); step ms = wall per step with the
queue kept full; gpu ms = time between a sync-ed start and the end of N queued steps.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    from optical_flow_amd import _lib
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import flow_net_spec, init_params
    from optical_flow_amd.train import KerasAdam, Trainer
    _lib.load()
    H, W, B = 384, 512, args.batch
    net = FlowNet(H, W, values=init_params(flow_net_spec(), 0))
    trainer = Trainer(net, KerasAdam(net.store), LossLayer())
    batch = torch.from_numpy(synthetic_batch(B, H, W, seed=1234)).cuda()
    for i in range(3):
        trainer.train_step(batch, i)
    torch.cuda.synchronize()
    enq = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        a = time.perf_counter()
        trainer.train_step(batch, 3 + i)
        enq.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("enqueue ms/step: mean %.3f min %.3f max %.3f" % (
        1e3 * sum(enq) / len(enq), 1e3 * min(enq), 1e3 * max(enq)))
    print("host loop %.3f ms/step, wall %.3f ms/step" % (1e3 * (t1 - t0) / args.steps,
                                                           1e3 * (t2 - t0) / args.steps))


if __name__ == "__main__":
    main()
