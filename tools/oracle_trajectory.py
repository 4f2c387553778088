"""Training trajectory of the CPU oracle from bench.py's exact start.

python tools/oracle_trajectory.py --steps 26 --dtype float32 --out profiles/r4_oracle_traj_f32.jsonl

Same weights (init_params(flow_net_spec(), 0)), same batch (synthetic_batch(B, H, W, seed=1234)),
same optimizer (Keras Adam, lr 1e-4, train.py:34) as bench.py; one line per step with the loss
and the mean / max |flow| per pyramid level of that step's forward (the weights before the
update, like train.py:47-61 returns them).  bench.py runs warmup + 1 (untimed timing step) +
steps train steps from this start: 26 at --steps 20 --warmup 5.  Oracle = test infrastructure:
this is a checker run on the host, never part of the product path.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ref_flow as R                                     # noqa: E402
from optical_flow_amd.data import synthetic_batch                    # noqa: E402
from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=26)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", choices=["float32", "float64"], default="float32")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    dt = getattr(torch, args.dtype)
    vals = init_params(flow_net_spec(levels=4), 0)
    p = {k: torch.tensor(v, dtype=dt) for k, v in vals.items()}
    x = torch.tensor(synthetic_batch(args.batch, args.height, args.width, seed=1234), dtype=dt)
    blocks = list(encoder_blocks(4))
    opt = R.KerasAdam()
    with open(args.out, "w") as f:
        for s in range(args.steps):
            t0 = time.time()
            loss, flows, _ = R.train_step(x, p, blocks, opt)
            rec = {"step": s, "loss": float(loss),
                   "flow_abs_mean": [round(float(fl.abs().mean()), 6) for fl in flows],
                   "flow_abs_max": [round(float(fl.abs().max()), 4) for fl in flows],
                   "dtype": args.dtype, "sec": round(time.time() - t0, 1)}
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
