#!/usr/bin/env python
"""Training throughput of the MI355X-native optical-flow hot path (BASELINE.json metric:
image-pairs/sec training, 384x512, batch 8 per GPU, at 1/2/4/8 MI355X; EPE vs ref).

One step = forward (Siamese encoder + 4 flow modules) + photometric loss + backward + (N>1:
RCCL all-reduce of gradient buckets, overlapped with the backward) + Keras-Adam update, on a
synthetic batch resident in HBM.  Launch: ``python bench.py`` (N=1) or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.

Prints ONE JSON line (rank 0) with the contract fields plus:
  roofline      -- dominant kernel (the conv instance with the largest total time) measured
                   with a hipEvent pair around every conv launch of the timed steps, on the
                   stream it is launched on: achieved = algorithmic FLOPs / launch duration,
                   vs the MFMA peak of the dtype.
  cpu_baseline  -- the CPU oracle (reference semantics restated in torch-CPU fp32) timed on
                   this host's usable cores on the bench batch (B=8 at 384x512: 1 untimed +
                   3 timed steps, capped at 60 s), rank 0 only.
  parity        -- EPE / loss error between the HIP path and that oracle run on the same
                   batch and initial weights.
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: f32 MFMA = f32 vector peak (spec)
MODE_NAMES = {0: "fwd", 1: "dgrad", 2: "wgrad"}
TILE_TEMPLATE = {0: "128, 128, 2, 2", 1: "128, 96, 4, 1", 2: "256, 64, 4, 1", 3: "256, 32, 4, 1",
                 7: "narrow"}
NARROW_SYMBOLS = {0: "oflow::narrow_fwd_kernel(oflow::NarrowArgs)",
                  1: "oflow::narrow_dgrad_kernel(oflow::NarrowArgs)",
                  2: "oflow::narrow_wgrad_kernel(oflow::NarrowArgs)"}


BF16_MFMA_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def kind_parts(kind):
    """timing kind -> (mode, tile config, family): f32 GEMMs mode*8+cfg (narrow VALU cfg 7),
    f32 halo-tiled wgrad 32 + mode*8 + cfg,
    bf16 implicit GEMMs 64 + mode*8 + cfg, bf16 halo-tiled 3x3 96 + mode*8 + cfg,
    fp32 on the split-bf16 halo-tiled 3x3 kernels 128 + mode*8 + cfg, on the split-bf16
    implicit GEMM (other shapes) 160 + mode*8 + cfg (optical_flow_amd/csrc/conv_f32.hip)."""
    if kind >= 304:                               # conv_wgrad_b16i (bf16 images)
        return 2, kind - 304, "wgrad_b16i"
    if kind >= 288:                               # conv_halo_b16 (bf16 images) fwd / dgrad
        return (kind - 288) // 8, (kind - 288) % 8, "halo_b16"
    if kind == KIND_STEM_X3:
        return 0, 0, "stem_x3"
    if kind == KIND_STEM_WG_X3:
        return 2, 0, "stem_x3"
    if kind == KIND_STEM_B16:
        return 0, 0, "stem_b16"
    if kind == KIND_STEM_WG_B16:
        return 2, 0, "stem_b16"
    if kind >= 240:                               # conv_gemm_x3 / conv_wgrad_x3, one plane (bf16)
        return (kind - 240) // 8, (kind - 240) % 8, "gemm_b16"
    if kind >= 224:                               # conv_tile_ws (warp-specialised bf16 3x3)
        return (kind - 224) // 8, (kind - 224) % 8, "tile_ws"
    if kind >= 216:                               # conv_wgrad_tile_b16 (x3b configs, 1 plane)
        return 2, kind - 216, "wgrad_b16"
    if kind >= 192:                               # conv_tile_b16 (bf16 on the x3 structure)
        return (kind - 192) // 8, (kind - 192) % 8, "tile_b16"
    fam = ("gemm_x3" if kind >= 160 else "tile_x3" if kind >= 128 else "tile_bf16" if kind >= 96 else
           "bf16" if kind >= 64 else
           "tile_f32" if kind >= 32 else "f32")
    if fam == "tile_x3" and kind >= 152:          # conv_wgrad_tile_x3b configs 8+ (cfg 4 of
        return 2, 8 + kind - 152, fam             # the C dispatch: 32 x 64 channel blocks)
    return (kind % 32) // 8, kind % 8, fam


TILE_BN = {0: "128, 2, 2", 1: "96, 4, 1", 2: "64, 2, 2", 3: "32, 4, 1", 4: "128, 4, 2"}
TILE_TH = {0: 4, 1: 4, 2: 4, 3: 4, 4: 8}                # conv_tile_bf16 output tile rows
X3_BN = {0: "128, 4, 2", 1: "96, 2, 3", 2: "64, 4, 2", 3: "32, 4, 1",   # conv_tile_x3 waves
         4: "128, 2, 2", 5: "96, 4, 3", 6: "128, 2, 4", 7: "64, 4, 1"}
X3_TH = {0: 8, 1: 4, 2: 4, 3: 4, 4: 4, 5: 8, 6: 4, 7: 8}                       # and tile rows
X3_NB = {4: 1, 7: 1}                                                           # single-buffered B
GX3 = {0: "128, 128, 4, 2", 1: "256, 64, 8, 1"}   # conv_gemm_x3<BM, BN, WAVES_M, WAVES_N>
GX3_WG = {0: "128, 128, 4, 2", 1: "128, 64, 4, 2"}  # conv_wgrad_x3<BM, BN, WAVES_M, WAVES_N>
X3_WGT = {0: "1, 4, 3, 8", 1: "1, 3, 3, 8", 2: "2, 2, 3, 4", 3: "2, 1, 3, 4",   # conv_wgrad_tile_x3<CI, CO, R, rows>
          4: "2, 4, 8, 1", 5: "2, 3, 8, 1", 6: "4, 2, 4, 1", 7: "4, 1, 4, 1",  # conv_wgrad_tile_x3b<CI, CO, rows, MI>
          8: "2, 2, 8, 1"}


WGT_WAVES = {0: "1, 4", 2: "2, 2"}   # conv_wgrad_tile_bf16<WAVES_CI, WAVES_CO>
WS_BN = {0: "128, 8, 2, 2", 1: "96, 8, 2, 2"}   # conv_tile_ws<BN, TH, CWM, CWN>
B16_WGT = {0: "2, 4, 8", 1: "2, 3, 8", 2: "4, 2, 4", 3: "4, 1, 4", 4: "2, 2, 8"}   # conv_wgrad_tile_b16


def conv_math(precision):
    """How the convs compute (the dtype field names the arithmetic type, fp32 or bf16)."""
    from optical_flow_amd import ops
    if precision == "bf16":
        return "bf16 MFMA operands, fp32 accumulation (flow convs cout<=4: fp32 VALU)"
    if ops.F32_SPLIT:
        return ("fp32: every conv with >= 16 input channels (3x3 stride-1 halo tiles; stride-2 "
                "and 1x1 implicit GEMMs) fwd/dgrad/wgrad on bf16 MFMA with an exact 3-term "
                "operand split (6 products, fp32 accumulation; error vs fp64 at fp32-MFMA level, "
                "test_conv_x3_accuracy / test_conv_gemm_x3_accuracy); the 3-channel stem's "
                "forward and weight gradient on their own split-bf16 kernels (conv_stem_x3, "
                "conv_wgrad_stem_x3), the Cout<=4 flow convs on fp32 VALU")
    return "fp32 MFMA (flow convs cout<=4: fp32 VALU)"


KIND_STEM_X3 = 184   # conv_stem_x3 (the 7x7 stride-2 stem forward on the split-bf16 MFMA)
KIND_STEM_WG_X3 = 185   # conv_wgrad_stem_x3 (its weight gradient)
KIND_STEM_B16 = 186     # conv_stem_x3<32, 1> (the bf16 stem forward, one plane)
KIND_STEM_WG_B16 = 187  # conv_wgrad_stem_x3<1> (its bf16 weight gradient)


HALO_B16 = {0: "128, 4, 2", 1: "96, 4, 2", 2: "64, 8, 1", 3: "32, 8, 1"}  # conv_halo_b16<BN, waves>
HALO_PERSIST = False   # of_set_tuning key 24 = 1 (set from --tune in main)
WGRAD_B16I = {0: "2, 4", 1: "4, 2", 2: "4, 1"}                          # conv_wgrad_b16i<waves>


def kind_name(kind):
    mode, cfg, fam = kind_parts(kind)
    if fam == "halo_b16":
        return "%s_halo_b16<%s>" % (MODE_NAMES[mode], HALO_B16[cfg])
    if fam == "wgrad_b16i":
        return "wgrad_b16i<%s>" % WGRAD_B16I[cfg]
    if fam == "stem_x3":
        return "wgrad_stem_x3" if mode == 2 else "fwd_stem_x3"
    if fam == "stem_b16":
        return "wgrad_stem_b16" if mode == 2 else "fwd_stem_b16"
    sfx = {"f32": "", "bf16": "_bf16", "tile_bf16": "_tile_bf16", "tile_f32": "_tile_f32",
           "tile_x3": "_tile_x3", "gemm_x3": "_gemm_x3", "tile_b16": "_tile_b16",
           "wgrad_b16": "", "tile_ws": "_tile_ws", "gemm_b16": "_gemm_b16"}[fam]
    if fam == "tile_ws":
        return "%s%s<%s>" % (MODE_NAMES[mode], sfx, WS_BN[cfg])
    if fam == "tile_b16":
        return "%s%s<%s, %d>" % (MODE_NAMES[mode], sfx, X3_BN[cfg], X3_TH[cfg])
    if fam == "wgrad_b16":
        return "wgrad_tile_b16<%s>" % B16_WGT[cfg]
    if fam in ("gemm_x3", "gemm_b16"):
        return "%s%s<%s>" % (MODE_NAMES[mode], sfx, (GX3_WG if mode == 2 else GX3)[cfg])
    if fam in ("tile_bf16", "tile_f32", "tile_x3") and mode == 2:
        if fam == "tile_x3" and cfg >= 4:
            sfx = "_tile_x3b"
        return "wgrad%s<%s>" % (sfx, X3_WGT[cfg] if fam == "tile_x3" else WGT_WAVES[cfg])
    if fam == "tile_x3":
        return "%s%s<%s, %d>" % (MODE_NAMES[mode], sfx, X3_BN[cfg], X3_TH[cfg])
    return "%s%s<%s>" % (MODE_NAMES[mode], sfx, (TILE_BN if fam == "tile_bf16"
                                                 else TILE_TEMPLATE)[cfg])


def kernel_symbol(kind):
    """rocprofv3 name of the conv kernel instance behind a timing kind."""
    mode, cfg, fam = kind_parts(kind)
    if fam == "halo_b16":    # last template argument: the persistent form (key 24, default off)
        return ("void oflow::(anonymous namespace)::conv_halo_b16<%s, %d, 16, 32, %s>"
                "(oflow::GemmArgs)" % (HALO_B16[cfg], mode, "true" if HALO_PERSIST else "false"))
    if fam == "wgrad_b16i":
        return "void oflow::(anonymous namespace)::conv_wgrad_b16i<%s>(oflow::GemmArgs)" % WGRAD_B16I[cfg]
    if fam == "stem_x3":
        if mode == 2:
            return "void oflow::conv_wgrad_stem_x3<3, false>(oflow::GemmArgs)"
        return "void oflow::conv_stem_x3<32, 3>(oflow::GemmArgs, int)"   # of_set_tuning key 8 default
    if fam == "stem_b16":
        if mode == 2:
            return "void oflow::conv_wgrad_stem_x3<1, false>(oflow::GemmArgs)"
        return "void oflow::conv_stem_x3<32, 1>(oflow::GemmArgs, int)"
    if cfg == 7 and fam == "f32":
        return NARROW_SYMBOLS[mode]
    if fam == "tile_b16":
        return "void oflow::conv_tile_b16<%s, %d, %d>(oflow::GemmArgs)" % (X3_BN[cfg], mode,
                                                                            X3_TH[cfg])
    if fam == "wgrad_b16":
        return "void oflow::conv_wgrad_tile_b16<%s>(oflow::GemmArgs)" % B16_WGT[cfg]
    if fam == "tile_ws":
        return "void oflow::conv_tile_ws<%s, %d>(oflow::GemmArgs)" % (WS_BN[cfg], mode)
    if fam in ("gemm_x3", "gemm_b16"):           # (the plane count NP: 3 split, 1 bf16)
        np_ = 3 if fam == "gemm_x3" else 1
        if mode == 2:
            return "void oflow::conv_wgrad_x3<%s, %d>(oflow::GemmArgs)" % (GX3_WG[cfg], np_)
        # (RING = 2: the DMA ring of of_set_tuning key 30 = 2, the default)
        return "void oflow::conv_gemm_x3<%s, %d, %d, 2>(oflow::GemmArgs)" % (GX3[cfg], mode, np_)
    if fam in ("tile_bf16", "tile_f32", "tile_x3") and mode == 2:
        # the bf16 form prints its defaulted fragment-prefetch flag too (PF = 1, key 17)
        return "void oflow::conv_wgrad_%s<%s%s>(oflow::GemmArgs)" % (
            fam + ("b" if fam == "tile_x3" and cfg >= 4 else ""),
            X3_WGT[cfg] if fam == "tile_x3" else WGT_WAVES[cfg],
            ", 1" if fam == "tile_bf16" else "")
    if fam in ("tile_bf16", "tile_x3"):
        if fam == "tile_x3":
            # the demangled name prints the defaulted NB too (conv_tile_x3<..., TH, NB>)
            return "void oflow::conv_tile_x3<%s, %d, %d, %d>(oflow::GemmArgs)" % (
                X3_BN[cfg], mode, X3_TH[cfg], X3_NB.get(cfg, 2))
        # (with its defaulted fragment-prefetch flag, PF = 1, of_set_tuning key 20)
        return "void oflow::conv_tile_bf16<%s, %d, %d, 1>(oflow::GemmArgs)" % (TILE_BN[cfg], mode,
                                                                               TILE_TH[cfg])
    if fam == "bf16" and mode == 2:
        return "void oflow::conv_wgrad_bf16<%s>(oflow::GemmArgs)" % TILE_TEMPLATE[cfg]
    return "void oflow::conv_gemm_%s<%s, %d>(oflow::GemmArgs)" % (fam, TILE_TEMPLATE[cfg], mode)


def gflop_per_pair(H, W, max_disp=3, levels=4):
    """Algorithmic training FLOPs per image pair (SURVEY.md §8 d): every conv's fwd + dgrad +
    wgrad (2 FLOP/MAC, logical channels, TF-'same' output sizes) minus the stem dgrad, plus
    3x the cost-volume forward."""
    from optical_flow_amd.params import ENC_CHANNELS, HEAD_WIDTHS, encoder_blocks, head_cin
    macs = 0.0
    h, w = H // 2, W // 2
    stem = 2 * h * w * 7 * 7 * 3 * 64             # both Siamese branches
    macs += 2 * stem                               # fwd + wgrad (no input grad for images)
    hh, ww = h // 2, w // 2
    for prefix, cin, cout, stride, proj in encoder_blocks(levels):
        ho, wo = hh // stride, ww // stride
        m = 2 * ho * wo                            # two branches
        macs += 3 * m * 9 * cin * cout             # conv_a
        macs += 3 * m * 9 * cout * cout            # conv_b
        if proj:
            macs += 3 * m * cin * cout
        hh, ww = ho, wo
    corr = 0.0
    for level in range(levels):
        s = (1 << levels) >> level
        ph, pw = H // s, W // s
        cin = head_cin(level, max_disp, levels)
        for cout in HEAD_WIDTHS:
            macs += 3 * ph * pw * 9 * cin * cout
            cin = cout
        c = ENC_CHANNELS[levels - 1 - level]
        corr += 2.0 * ph * pw * (2 * max_disp + 1) ** 2 * c
    return (2 * macs + 3 * corr) / 1e9


def host_cores():
    """(cores this process may use, CPUs the host reports).  On the GPU box os.cpu_count()
    shows the whole machine while the job gets a share of it (a cgroup CPU quota, and
    OMP_NUM_THREADS set to that share): the usable count is the smallest of the affinity
    mask, the quota and OMP_NUM_THREADS."""
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        usable = min(usable, int(omp))
    return usable, total


def cpu_baseline(batch_np, vals, steps=3, precision="fp32", levels=4, max_s=60.0):
    """The oracle's train_step (torch CPU fp32, the reference semantics restated) on the
    bench's own batch (SURVEY.md §8 d: B=8 at 384x512), all usable host cores: 1 untimed step
    (which also gives the reference flows / loss at the initial weights for the parity
    probe), then ``steps`` timed steps, stopping early after ``max_s`` seconds.  Returns
    (pairs/s, threads, host CPUs, timed steps, flows_at_init, loss_at_init).  With precision
    "bf16" the reference outputs come from the oracle with the build's bf16 operand rounding;
    the timed steps are always the fp32 reference semantics."""
    from oracle import ref_flow as R
    from optical_flow_amd.params import encoder_blocks
    threads, total = host_cores()
    torch.set_num_threads(threads)
    p = {k: torch.tensor(v) for k, v in vals.items()}
    blocks = list(encoder_blocks(levels))
    x = torch.tensor(batch_np)
    R.set_conv_precision(precision)
    try:
        loss0, flows0, _ = R.train_step(x, p, blocks, None)  # warm-up + reference outputs
    finally:
        R.set_conv_precision("fp32")
    opt = R.KerasAdam()
    t0 = time.time()
    n = 0
    while n < steps:
        R.train_step(x, p, blocks, opt)
        n += 1
        if time.time() - t0 > max_s:
            break
    dt = time.time() - t0
    return n * x.shape[0] / dt, threads, total, n, flows0, float(loss0)


def final_parity(pair_np, params, flows_hip, precision="fp32", levels=4):
    """EPE / relative error of the HIP forward against the oracle's forward (float64; for bf16
    with the build's bf16 operand rounding) on one pair at the weights the timed steps ended
    with -- the parity probe above checks only the initial weights."""
    from oracle import ref_flow as R
    from optical_flow_amd.params import encoder_blocks
    p = {k: v.double() for k, v in params.items()}
    R.set_conv_precision(precision)
    try:
        with torch.no_grad():
            fo = R.flow_net(torch.tensor(pair_np, dtype=torch.float64), p,
                            list(encoder_blocks(levels)))
    finally:
        R.set_conv_precision("fp32")
    epe = [float((a.double() - b).norm(dim=-1).mean()) for a, b in zip(flows_hip, fo)]
    rel = [float((a.double() - b).abs().max() / b.abs().max()) for a, b in zip(flows_hip, fo)]
    return {"epe": [round(e, 6) for e in epe], "flow_rel_inf": [float("%.3e" % r) for r in rel],
            "note": "HIP forward vs the oracle's, pair 0 of the bench batch, the weights after "
                    "the last timed step"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8, help="pairs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--timing-steps", type=int, default=2,
                    help="steps whose conv launches carry hipEvent pairs: the last ones of the "
                         "timed region (or, with --roofline-window extra, extra steps)")
    ap.add_argument("--roofline-window", choices=["timed", "extra"], default="timed",
                    help="timed: per-launch hipEvents over the timed steps (default); extra: "
                         "separate instrumented steps with every conv on one stream")
    ap.add_argument("--levels", type=int, choices=[4, 5], default=4,
                    help="5: the reference's commented-out 5th pyramid level (model.py:24-25)")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="fp32: config 2 (headline); bf16: configs 3-5 conv contractions on "
                         "bf16 MFMA with fp32 accumulation")
    ap.add_argument("--tune", default=None, help="key=value[,...] of_set_tuning (experiments)")
    ap.add_argument("--graph", type=int, choices=[0, 1], default=0,
                    help="1: capture the train step once as a HIP graph and replay it (the "
                         "timed steps); 0 (default, measured faster: DESIGN.md §4): eager "
                         "launches through the Python glue")
    ap.add_argument("--side-stream", type=int, choices=[0, 1], default=1,
                    help="1: weight-gradient kernels on a second HIP stream (ops.side_stream)")
    ap.add_argument("--main-prio", type=int, choices=[0, 1],
                    default=int(os.environ.get("OFLOW_MAIN_PRIO", "0")),
                    help="1: run the step on a high-priority HIP stream, so the hardware "
                         "dispatches its workgroups ahead of the side streams' (weight "
                         "gradients, the cost volume's df1) when both have work queued")
    ap.add_argument("--deterministic", type=int, choices=[0, 1],
                    default=int(os.environ.get("OFLOW_DETERMINISTIC", "1")),
                    help="1 (default): the deterministic warp backward (window gather / int64 "
                         "fixed point, ops.DETERMINISTIC); 0: the float-atomic warp_bwd_gather")
    args = ap.parse_args()

    from optical_flow_amd import _lib, ops
    ops.SIDE_STREAM_WGRAD = bool(args.side_stream)
    ops.set_deterministic(bool(args.deterministic))
    if args.tune:
        for kv in args.tune.split(","):
            k, v = kv.split("=")
            _lib.lib().of_set_tuning(int(k), int(v))
            if int(k) == 24:
                global HALO_PERSIST
                HALO_PERSIST = int(v) != 0
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.dist import init_from_env
    from optical_flow_amd.loss import LossLayer
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import flow_net_spec, init_params
    from optical_flow_amd.train import KerasAdam, Trainer

    rank, world, local = init_from_env()
    torch.cuda.set_device(local)
    if args.main_prio:
        torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    _lib.load()
    H, W, B = args.height, args.width, args.batch
    vals = init_params(flow_net_spec(levels=args.levels), 0)   # identical weights on all ranks
    net = FlowNet(H, W, values=vals, precision=args.precision, levels=args.levels)
    trainer = Trainer(net, KerasAdam(net.store), LossLayer())
    batch = torch.from_numpy(synthetic_batch(B, H, W, seed=1234, rank=rank)).cuda()

    # ---- parity probe: HIP forward on the whole bench batch with the initial weights -----
    with torch.no_grad():
        flows_hip = [f.cpu() for f in net(batch)]
        loss_hip = float(LossLayer()(batch, [f.cuda() for f in flows_hip]))

    # ---- training throughput --------------------------------------------------------------
    # The roofline timing is taken live in the timed region: over its last --timing-steps
    # steps each launch of the dominant conv kernel is bracketed by a hipEvent pair on the
    # stream it is launched on (one-shot of_timing_enable(2) from ops._tag), so its durations
    # are those of the measured run.  Which kernel dominates, and the per-kernel table, come
    # from one untimed step after the warm-up with every conv launch timed (event pairs around
    # all ~130 conv launches of a step cost ~6 % of that step; around the dominant kernel's
    # ~14, ~0.5 %).
    lib = _lib.lib()
    for i in range(args.warmup):
        trainer.train_step(batch, i)
    torch.cuda.synchronize()
    live = args.roofline_window == "timed"
    prof_per, prof_only, alone = {}, None, {}
    if live:
        ops.TIMING_TAGS = []
        lib.of_timing_read(0, None, None, None)
        lib.of_timing_enable(1)
        trainer.train_step(batch, 20_000)
        torch.cuda.synchronize()
        lib.of_timing_enable(0)
        ptags, ops.TIMING_TAGS = ops.TIMING_TAGS, None
        pcap = 16384
        pk, pf, pm = (C.c_int * pcap)(), (C.c_double * pcap)(), (C.c_float * pcap)()
        pn = lib.of_timing_read(pcap, pk, pf, pm)
        for i in range(pn):
            tf, tm, cnt = prof_per.get(pk[i], (0.0, 0.0, 0))
            prof_per[pk[i]] = (tf + pf[i], tm + pm[i], cnt + 1)
        pkinds = [pk[i] for i in range(pn)]
        # The same table with every kernel alone on the chip: one more untimed step with the
        # side streams off (weight gradients, BN reductions and forward projections on the
        # main stream).  In the step above the input-gradient convs share the chip with the
        # side stream's weight gradients and BN reductions, which stretches their event spans;
        # this one separates kernel efficiency from that overlap (same thermal state).
        side0, proj0 = ops.SIDE_STREAM_WGRAD, ops.PROJ_SIDE
        ops.SIDE_STREAM_WGRAD = ops.PROJ_SIDE = False
        lib.of_timing_read(0, None, None, None)
        lib.of_timing_enable(1)
        trainer.train_step(batch, 20_001)
        torch.cuda.synchronize()
        lib.of_timing_enable(0)
        ops.SIDE_STREAM_WGRAD, ops.PROJ_SIDE = side0, proj0
        for i in range(lib.of_timing_read(pcap, pk, pf, pm)):
            tf, tm, cnt = alone.get(pk[i], (0.0, 0.0, 0))
            alone[pk[i]] = (tf + pf[i], tm + pm[i], cnt + 1)
        # The dominant kernel: the largest per-step time with every kernel alone (its own cost;
        # in the step above, a kernel's span also counts the side-stream work it overlaps, and
        # the two largest instances trade places run to run); its launches are then timed live
        # in the timed region.
        if prof_per and len(ptags) == pn and not os.environ.get("OFLOW_TIMING_DUMP"):
            by = alone if alone else prof_per
            pdom = max(by, key=lambda k: by[k][1])
            prof_only = {ptags[i] for i in range(pn) if pkinds[i] == pdom}
    torch.cuda.synchronize()
    graphed = None
    if args.graph:
        # The whole step captured once as a HIP graph (Trainer.graphed) and replayed.  Event
        # pairs captured as hipEventRecordExternal nodes around the dominant kernel's launches
        # read back out of order (negative spans, measured), so in this mode the roofline
        # durations are those of the fully timed eager step after the warm-up.
        graphed = trainer.graphed(batch, warmup=1)
        for _ in range(2):                              # upload + first replays, untimed
            graphed()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timed_from = max(0, args.steps - args.timing_steps)      # the last timing_steps steps
    first = None                    # (loss, flows) of the first timed step, read afterwards
    t0 = time.perf_counter()
    for i in range(args.steps):
        if graphed is not None:
            loss, flows = graphed()
            if i == 0:
                first = (loss.clone(), [f.clone() for f in flows])
            continue
        if live and i == timed_from:
            ops.TIMING_TAGS = []
            if prof_only is not None:
                ops.TIMING_ONLY = prof_only
            else:                                   # fallback: every conv launch
                lib.of_timing_enable(1)
        loss, flows = trainer.train_step(batch, args.warmup + i)
        if i == 0:
            first = (loss, flows)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if live:
        ops.TIMING_ONLY = None
        lib.of_timing_enable(0)
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64)
    if world > 1:     # control plane (gloo); the gradients went over the C-ABI RCCL comm
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed)
    pairs = world * B * args.steps
    value = pairs / elapsed
    final_loss = float(loss)
    # The training state the timed steps ran in (the warp backward's work depends on where
    # the flows send samples: clipped borders): loss and mean / max |flow| per level at the
    # first and the last timed step.  From this start the reference semantics themselves
    # diverge at the coarse levels within ~20 steps (profiles/r4_oracle_traj_f32.jsonl).
    flow_abs = [[round(float(f.abs().mean()), 4), round(float(f.abs().max()), 3)] for f in flows]
    timed_state = {"first": {"loss": float(first[0]),
                             "flow_abs_mean": [round(float(f.abs().mean()), 4) for f in first[1]]},
                   "last": {"loss": final_loss,
                            "flow_abs_mean": [round(float(f.abs().mean()), 4) for f in flows]},
                   "train_steps_before_first": args.warmup + (2 if live else 0) +
                                               (3 if graphed is not None else 0)}

    # ---- dominant-kernel roofline ------------------------------------------------------------
    nsteps = args.steps - timed_from
    if not live:   # --roofline-window extra: separate instrumented steps, convs on one stream
        nsteps = args.timing_steps
        ops.TIMING_TAGS = []
        ops.SIDE_STREAM_WGRAD = False
        lib.of_timing_enable(1)
        for i in range(args.timing_steps):
            trainer.train_step(batch, 10_000 + i)
        torch.cuda.synchronize()
        lib.of_timing_enable(0)
        ops.SIDE_STREAM_WGRAD = bool(args.side_stream)
    tags, ops.TIMING_TAGS = ops.TIMING_TAGS, None
    cap = 16384
    kinds = (C.c_int * cap)()
    flops = (C.c_double * cap)()
    ms = (C.c_float * cap)()
    n = lib.of_timing_read(cap, kinds, flops, ms)
    per = {}
    for i in range(n):
        k = kinds[i]
        tf, tm, cnt = per.get(k, (0.0, 0.0, 0))
        per[k] = (tf + flops[i], tm + ms[i], cnt + 1)
    if graphed is not None:          # graph mode: the fully timed eager step (see above)
        per, nsteps = dict(prof_per), 1
    if os.environ.get("OFLOW_TIMING_DUMP") and rank == 0 and len(tags) == n:
        with open(os.environ["OFLOW_TIMING_DUMP"], "w") as f:
            json.dump([{"layer": tags[i][0], "kind": kinds[i], "gflop": flops[i] / 1e9,
                        "ms": ms[i]} for i in range(n)], f)
    dom = max(per, key=lambda k: per[k][1]) if per else None
    # per-kernel table and all-conv rate: the fully timed untimed step (one step), when the
    # timed region timed the dominant kernel only
    table, tsteps = (prof_per, 1) if (live and prof_only is not None) else (per, max(nsteps, 1))
    roof = None
    conv_ms_step = sum(v[1] for v in table.values()) / tsteps
    if dom is not None:
        tf, tm, cnt = per[dom]
        achieved = tf / (tm * 1e-3) / 1e12
        sym = kernel_symbol(dom)
        traffic = mfma_busy = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                db = json.load(f)
            pmc = db.get("entries", {}).get("%s:%dx%dx%d" % (args.precision, H, W, B), {})
            same_math = args.precision != "fp32" or pmc.get("f32_split", True) == ops.F32_SPLIT
            if same_math and sym in pmc.get("kernels", {}):
                traffic = pmc["kernels"][sym].get("hbm_bytes_per_launch")
                # SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles), tools/pmc_mfma.py
                mfma_busy = pmc["kernels"][sym].get("mfma_busy")
        allconv = sum(v[0] for v in table.values()) / (sum(v[1] for v in table.values()) * 1e-3) / 1e12
        fam = kind_parts(dom)[2]
        # the split kernel spends six bf16 MFMAs per fp32 product: its ceiling is 1/6 of bf16
        peak = (FP32_MFMA_PEAK_TFLOPS if fam in ("f32", "tile_f32") else
                round(BF16_MFMA_PEAK_TFLOPS / 6, 1) if fam in ("tile_x3", "gemm_x3", "stem_x3")
                else BF16_MFMA_PEAK_TFLOPS)
        roof = {"bound": "mfma", "kernel": sym, "achieved": round(achieved, 2),
                "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "mfma_busy": mfma_busy,
                "launches_per_step": cnt // max(nsteps, 1),
                "window": ("one fully timed eager step after the warm-up (the timed region "
                           "replayed the captured graph)" if graphed is not None else
                           ("timed region, %d steps (the dominant kernel's launches timed; "
                            "per_kernel from one fully timed step after the warm-up, "
                            "per_kernel_alone from one with the side streams off, which "
                            "picks the dominant kernel)" % nsteps)
                           if live and prof_only is not None else
                           ("timed region, %d steps" % nsteps) if live else
                           ("%d extra steps, convs on one stream" % nsteps)),
                "avg_launch_ms": round(tm / cnt, 4), "gflop_per_launch": round(tf / cnt / 1e9, 3),
                "all_conv_gemm_tflops": round(allconv, 2),
                "per_kernel": {kind_name(k):
                               {"launches_per_step": v[2] // tsteps,
                                "ms_per_step": round(v[1] / tsteps, 3),
                                "tflops": round(v[0] / (v[1] * 1e-3) / 1e12, 2)}
                               for k, v in sorted(table.items())}}

    if roof is not None and alone:
        roof["all_conv_gemm_tflops_alone"] = round(
            sum(v[0] for v in alone.values()) / (sum(v[1] for v in alone.values()) * 1e-3) / 1e12, 2)
        roof["per_kernel_alone"] = {
            kind_name(k): {"launches_per_step": v[2], "ms_per_step": round(v[1], 3),
                           "tflops": round(v[0] / (v[1] * 1e-3) / 1e12, 2)}
            for k, v in sorted(alone.items())}

    # ---- parity probe at the final weights: HIP forward of one pair (the oracle runs after
    # the timed region, below) -------------------------------------------------------------
    with torch.no_grad():
        flows_fin = [f.cpu() for f in net(batch[:1])]
    params_fin = {k: v.detach().cpu() for k, v in net.store.params.items()}

    # ---- CPU baseline + EPE vs the oracle (rank 0 only) ----------------------------------
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:     # N=1 only (contract)
        cps, threads, host_cpus, nsteps_cpu, flows_ref, loss_ref = cpu_baseline(
            batch.cpu().numpy(), vals, args.cpu_steps, args.precision, args.levels)
        cpu = {"value": round(cps, 4), "unit": "image-pairs/s", "cores": threads,
               "threads": threads, "host_cpus": host_cpus, "kind": "port",
               "sample": "%d oracle train steps (torch-CPU fp32 restatement of the reference "
                         "semantics, Keras Adam included) on the bench batch, B=%d at %dx%d, "
                         "after 1 untimed step; %d threads = the cores this job may use (%d "
                         "CPUs on the host)" % (nsteps_cpu, B, H, W, threads, host_cpus)}
        epe = [float((a - b.float()).norm(dim=-1).mean()) for a, b in zip(flows_hip, flows_ref)]
        rel = [float((a - b.float()).abs().max() / b.abs().max()) for a, b in
               zip(flows_hip, flows_ref)]
        parity = {"epe": [round(e, 6) for e in epe], "flow_rel_inf": [float("%.3e" % r) for r in rel],
                  "loss_rel": float("%.3e" % (abs(loss_hip - loss_ref) / abs(loss_ref))),
                  "note": "HIP %s vs CPU oracle (%s operand rounding), the bench batch (B=%d) "
                          "and initial weights, flows [H/2 ... H/%d]" % (
                              args.precision, args.precision, B, 2 ** args.levels)}
        parity["final_weights"] = final_parity(batch[:1].cpu().numpy(), params_fin, flows_fin,
                                               args.precision, args.levels)

    gfp = gflop_per_pair(H, W, levels=args.levels)
    if rank == 0:
        out = {
            "metric": "image-pairs/sec training, %dx%d batch=%d per GPU" % (H, W, B),
            "value": round(value, 3),
            "unit": "image-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.precision == "fp32" else "bf16",
            "data": "synthetic (U[0,1)-mean pairs, image2 = shifted image1 + noise; resident in HBM)",
            "config": {"workload": "full model.py encoder-decoder + loss.py photometric loss, "
                                   "train step (fwd+bwd+Keras Adam)",
                       "height": H, "width": W, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": "dp%d" % world,
                       "params": sum(p.numel() for p in net.trainable_weights),
                       "conv_math": conv_math(args.precision),
                       "execution": ("HIP graph: the train step captured once, replayed per step"
                                     if graphed is not None else "eager launches"),
                       "warp_backward": "deterministic" if ops.DETERMINISTIC else "atomic",
                       **({"grad_allreduce": (
                           "C-ABI RCCL communicator (of_comm_*), self-tested at init"
                           if trainer.reducer.comm.kind == "rccl" else
                           "torch.distributed %s" % dist.get_backend(trainer.reducer.comm.group))}
                          if trainer.reducer is not None else {}),
                       **({"levels": args.levels} if args.levels != 4 else {})},
            "algorithmic_gflop_per_pair": round(gfp, 2),
            "model_tflops": round(gfp * value / 1e3, 2),
            "conv_ms_per_step": round(conv_ms_step, 3),
            "final_loss": final_loss,
            "flow_abs_mean_max": flow_abs,
            "timed_state": timed_state,
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
