"""How well-conditioned is the flow net's train step in bn_mode="training" (P5) against the
inference mode?  The CPU oracle run in float32 against itself in float64, same weights and
input: per-level flow gaps, loss gap and the gradient gaps (median / worst rel l2), plus the
minimum distance of any oracle sample coordinate to an integer (the warp's floor() kink) and
of any L1 residual to zero (the loss's |.| kink).  A gap that the fp32 ORACLE shows as well is
the conditioning of the step, not a HIP-kernel defect (tests/test_gpu_bn_train.py).

    python tools/bn_train_conditioning.py [--seeds 4321,23,...] [--wseed 21]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_flow as R  # noqa: E402
from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params, perturb_params  # noqa: E402


def _coord_dist(f):
    """min distance of a warp's sample coordinates (grid + flow, P1) to an integer"""
    h, w = f.shape[1], f.shape[2]
    ii, jj = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    pts = torch.stack([ii, jj], -1).double() + f
    frac = (pts - pts.floor())
    return float(torch.minimum(frac, 1 - frac).min())


def kinks(batch, flows):
    """(min distance of a sample coordinate to an integer, min |residual|) over the loss
    warps (loss.py:26) and the feature warps (model.py:93: the coarser level's flow upscaled,
    R.upscale_flow)."""
    dmin, rmin = 1.0, 1e9
    x = torch.tensor(batch, dtype=torch.float64)
    H, W = x.shape[1], x.shape[2]
    for s in range(len(flows) - 1):
        dmin = min(dmin, _coord_dist(R.upscale_flow(flows[s + 1])))
    for s, f in enumerate(flows):
        h, w = H >> (s + 1), W >> (s + 1)
        dmin = min(dmin, _coord_dist(f))
        r = R.resize_bilinear(x, h, w)
        res = r[..., :3] - R.warp_features(f, r[..., 3:])
        rmin = min(rmin, float(res.abs().min()))
    return dmin, rmin


def run(batch, vals, mode, dtype):
    p = {k: torch.tensor(v, dtype=dtype) for k, v in vals.items()}
    R.set_bn_mode(mode)
    try:
        loss, flows, grads = R.train_step(torch.tensor(batch, dtype=dtype), p,
                                          list(encoder_blocks()), None)
    finally:
        R.set_bn_mode("inference")
    return loss, flows, grads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="4321,23")
    ap.add_argument("--wseed", type=int, default=21)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--W", type=int, default=128)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--out-scale", type=float, default=1.0,
                    help="scale of every flow module's last conv (conv5 kernel and bias)")
    a = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count()))
    vals = perturb_params(init_params(flow_net_spec(), a.wseed), a.wseed + 1)
    for k in vals:
        if "/conv5/" in k:
            vals[k] = vals[k] * a.out_scale
    print("weights seed %d, flow-module conv5 x %g" % (a.wseed, a.out_scale))
    for seed in [int(s) for s in a.seeds.split(",")]:
        batch = synthetic_batch(a.B, a.H, a.W, seed=seed)
        for mode in ("inference", "training"):
            l64, f64, g64 = run(batch, vals, mode, torch.float64)
            l32, f32, g32 = run(batch, vals, mode, torch.float32)
            fr = [float((a_.double() - b).abs().max() / b.abs().max()) for a_, b in zip(f32, f64)]
            ge = sorted(float((g32[n].double() - g64[n]).norm() / g64[n].norm().clamp_min(1e-30))
                        for n in g64 if not n.endswith("/bias"))
            dmin, rmin = kinks(batch, f64)
            fmax = " ".join("%.1f" % float(f.abs().max()) for f in f64)
            print("seed %d %-9s max|flow| %s  loss rel %.1e  flows rel_inf %s  grads rel_l2 median %.1e "
                  "worst %.1e  | min coord-to-integer %.1e, min |residual| %.1e" % (
                      seed, mode, fmax, abs(float(l32) - float(l64)) / abs(float(l64)),
                      " ".join("%.1e" % e for e in fr), float(np.median(ge)), ge[-1], dmin, rmin),
                  flush=True)


if __name__ == "__main__":
    main()
