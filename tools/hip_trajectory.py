"""Training trajectory of the HIP path from bench.py's exact start (GPU).

python tools/hip_trajectory.py --steps 26 [--det] [--precision fp32] --out gpurun_out/traj.jsonl

Same weights, batch and optimizer as bench.py and tools/oracle_trajectory.py; one JSON line
per step: loss and mean / max |flow| per level of that step's forward (the weights before the
update).  --det runs the deterministic warp backward (ops.deterministic()), so two runs
print identical curves; --oracle-every K additionally runs the oracle's forward (float64, one
pair) on the current weights every K steps and reports the flow EPE / loss error, i.e. where
the two trajectories' states part.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=26)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--det", action="store_true")
    ap.add_argument("--oracle-every", type=int, default=0)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    from optical_flow_amd import _lib, ops
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params
    from optical_flow_amd.train import KerasAdam, Trainer
    _lib.load()
    ops.set_deterministic(args.det)
    H, W, B = args.height, args.width, args.batch
    vals = init_params(flow_net_spec(levels=4), 0)
    net = FlowNet(H, W, values=vals, precision=args.precision)
    trainer = Trainer(net, KerasAdam(net.store), LossLayer())
    batch_np = synthetic_batch(B, H, W, seed=1234)
    batch = torch.from_numpy(batch_np).cuda()
    blocks = list(encoder_blocks(4))
    with open(args.out, "w") as f:
        for s in range(args.steps):
            rec = {"step": s, "det": args.det, "precision": args.precision}
            if args.oracle_every and s % args.oracle_every == 0:
                from oracle import ref_flow as R
                p = {k: v.detach().double().cpu() for k, v in net.store.params.items()}
                with torch.no_grad():
                    fh = [fl.double().cpu() for fl in net(batch[:1])]
                    R.set_conv_precision(args.precision)
                    try:
                        fo = R.flow_net(torch.tensor(batch_np[:1], dtype=torch.float64), p, blocks)
                    finally:
                        R.set_conv_precision("fp32")
                rec["epe_vs_oracle_pair0"] = [round(float((a - b).norm(dim=-1).mean()), 6)
                                              for a, b in zip(fh, fo)]
            t0 = time.time()
            loss, flows = trainer.train_step(batch, s)
            torch.cuda.synchronize()
            rec.update({"loss": float(loss),
                        "flow_abs_mean": [round(float(fl.abs().mean()), 6) for fl in flows],
                        "flow_abs_max": [round(float(fl.abs().max()), 4) for fl in flows],
                        "sec": round(time.time() - t0, 3)})
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
