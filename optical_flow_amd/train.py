"""Mirror of the reference ``train.py`` driver (train.py:1-88).

``train_step(batch_imgs, step_count)`` keeps the reference's shape (train.py:47-61): forward
through the flow net, the photometric loss, gradients of the trainable weights, one Keras-Adam
update; returns ``(loss_value, flows)``.  Data: ``--kitti PATH`` reads KITTI raw pairs
through the native AsyncReader (data_reader.py; batches land in HBM already resized and
normalised), otherwise synthetic pairs with the reference value contract (data.py).
``--display-dir`` writes the every-10-batches display_training pictures (train.py:80-81) as
PNGs.  No TensorBoard writer (a JSONL step log instead).  Data parallelism (one process per
GPU, RCCL all-reduce of gradient buckets overlapped with the backward) is build-added; with
KITTI each rank reads its own seeded shuffle.

Run:  python -m optical_flow_amd.train --height 384 --width 512 --batch 8 --steps 20
      python -m optical_flow_amd.train --kitti /data/kitti_raw --epochs 20
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np
import torch

from . import ops
from ._lib import call
from .data import synthetic_batch
from .dist import GradBucketReducer, init_from_env
from .loss import LossLayer
from .model import FlowNet, build_flow_net


class KerasAdam:
    """tf.keras.optimizers.Adam (train.py:34): beta_1 0.9, beta_2 0.999, epsilon 1e-7,
    ResourceApplyAdam update with lr_t = lr*sqrt(1-b2^t)/(1-b1^t) (P13).  Two launches over
    the model's parameter arena: the step counter t and lr_t live in device memory
    (of_adam_keras_dev), so the same update also runs inside a captured HIP graph
    (Trainer.graphed).  ``learning_rate`` may be set between steps (train.py:69-70)."""

    def __init__(self, store, learning_rate=1e-4, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.store = store
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon
        dev = store.arena.device
        self.m = torch.zeros_like(store.arena)
        self.v = torch.zeros_like(store.arena)
        self._sched = torch.zeros(2, device=dev)              # [lr, lr_t of the last step]
        self._iter = torch.zeros(1, dtype=torch.int32, device=dev)
        self.learning_rate = learning_rate

    @property
    def learning_rate(self):
        return self._lr

    @learning_rate.setter
    def learning_rate(self, lr):
        self._lr = float(lr)
        self._sched[0].fill_(self._lr)

    @property
    def iterations(self):
        """Updates applied so far (device counter: replays of a captured step count too)."""
        return int(self._iter.item())

    def apply_gradients(self, grad_scale: float = 1.0):
        s = self.store
        call("of_adam_keras_dev", C.c_void_p(s.arena.data_ptr()),
             C.c_void_p(s.grad_arena.data_ptr()), C.c_void_p(self.m.data_ptr()),
             C.c_void_p(self.v.data_ptr()), s.numel, C.c_void_p(self._sched.data_ptr()),
             C.c_void_p(self._iter.data_ptr()), self.beta_1, self.beta_2, self.epsilon,
             grad_scale, ops._stream())
        s.version += 1       # packed conv weights are refreshed lazily on next use
        if getattr(s, "bn_guard", None) is not None:
            s.bn_guard.after_update(self._lr)


class Trainer:
    """Holds the model, optimizer, loss and (optional) DP reducer; ``train_step`` is the
    hot loop body of train.py:72-82."""

    def __init__(self, flow_net: FlowNet, optimizer: KerasAdam = None, loss_layer=None,
                 data_parallel: bool = None, comm=None):
        """data_parallel: sum the gradients over ranks before Adam (default: when a
        torch.distributed group of > 1 ranks exists).  comm: a communicator (comm.py), or
        "rccl" / "torch" to create one; default "rccl" for a GPU model (the C-ABI RCCL
        communicator over all ranks of the default group), "torch" otherwise."""
        self.flow_net = flow_net
        self.optimizer = optimizer or KerasAdam(flow_net.store)
        self.loss_layer = loss_layer or LossLayer()
        if data_parallel is None:
            data_parallel = comm is not None or (torch.distributed.is_initialized() and
                                                 torch.distributed.get_world_size() > 1)
        self.reducer = None
        if data_parallel:
            if comm is None or isinstance(comm, str):
                from .comm import make_comm
                dist = torch.distributed
                rank, world = ((dist.get_rank(), dist.get_world_size())
                               if dist.is_initialized() else (0, 1))
                kind = comm or os.environ.get("OFLOW_DP_COMM") or (
                    "rccl" if flow_net.store.arena.is_cuda else "torch")
                comm = make_comm(kind, rank, world)
            self.reducer = GradBucketReducer(flow_net.store, comm=comm)

    def train_step(self, batch_imgs, step_count=0):
        store = self.flow_net.store
        store.zero_grad()
        if self.reducer is not None:
            self.reducer.begin()
        flows = self.flow_net(batch_imgs)
        loss_value = self.loss_layer(batch_imgs, flows)
        loss_value.backward()
        scale = 1.0
        if self.reducer is not None:
            # bn_mode "training": the moving statistics this step updated on every rank are
            # averaged over the ranks (dist.GradBucketReducer.finish), so replicas stay equal
            bufs = store.buffers if getattr(self.flow_net, "bn_mode", "") == "training" else None
            scale = self.reducer.finish(buffers=bufs)
        self.optimizer.apply_gradients(grad_scale=scale)
        return loss_value.detach(), [f.detach() for f in flows]

    def graphed(self, batch_imgs, warmup: int = 2, capture_ctx=None):
        """The step captured once as a HIP graph over a static input batch (train.py:47-48
        traces train_step once as a tf.function; this is the MI355X counterpart): returns a
        GraphedStep whose call copies nothing and replays every kernel of forward, loss,
        backward, bucket all-reduce (RCCL) and Adam with no host work per launch.
        ``warmup`` eager steps run first (they train, like any step)."""
        return GraphedStep(self, batch_imgs, warmup, capture_ctx)


# The captured step replays on a HIGH-priority stream of its own (torch.cuda.Stream(priority=-1),
# ordered after and before the caller's stream).  The HIP runtime inside the torch wheel (ROCm
# 7.0.2 libamdhip64, which liboflow binds to in a torch process) assigns a graph executor's
# parallel streams at its first launch by skipping those on the launch stream's hardware queue,
# without bounds: when one of them shares that queue it reads past the end of its stream list
# and segfaults in hipGraphLaunch (native backtrace, and the subset that
# crashed passing with this change).  Which queue a stream gets depends on every stream the
# process made before (RCCL's included); high-priority streams take their queues from a set of
# their own, so the normal-priority parallel streams never share the launch stream's.
# OFLOW_GRAPH_REPLAY_PRIO overrides the priority ("none": replay on the caller's stream).
_RP = os.environ.get("OFLOW_GRAPH_REPLAY_PRIO", "-1")
REPLAY_PRIO = None if _RP == "none" else int(_RP)


class GraphedStep:
    """A captured Trainer.train_step.  ``batch`` is the static input: write the next batch
    into it (``load``) before calling.  Returns the static (loss, flows) tensors, overwritten
    by every replay."""

    def __init__(self, trainer: "Trainer", batch_imgs, warmup: int = 2, capture_ctx=None):
        """capture_ctx: optional context-manager factory entered around the capture only (the
        bench arms its kernel timing there)."""
        if trainer.reducer is not None and getattr(trainer.reducer.comm, "kind", "") != "rccl":
            raise RuntimeError("graph capture needs the RCCL communicator (gloo collectives "
                               "cannot be captured)")
        self.trainer = trainer
        self.batch = batch_imgs
        cur = torch.cuda.current_stream()
        s = torch.cuda.Stream()
        s.wait_stream(cur)
        with torch.cuda.stream(s):                   # warm-up off the default stream (torch
            for i in range(warmup):                  # capture rule), creates the side streams
                trainer.train_step(batch_imgs, i)
        cur.wait_stream(s)
        self.captures = 0
        self._rs = None
        self._capture(capture_ctx)

    def _capture(self, capture_ctx=None):
        self.graph = torch.cuda.CUDAGraph()
        with capture_ctx() if capture_ctx is not None else contextlib.nullcontext():
            with torch.cuda.graph(self.graph):
                self.loss, self.flows = self.trainer.train_step(self.batch)
        self.captures += 1

    def load(self, batch_imgs):
        self.batch.copy_(batch_imgs, non_blocking=True)

    def __call__(self, batch_imgs=None, step_count=0):
        """One replay.  The BN gamma guard (ops.BNZGuard) is driven from here: the captured
        step bakes in which BN layers store z, so every BNZGuard.EVERY replays the guard's
        min |gamma| check is launched after the replay (read back asynchronously), and when a
        check flags a new layer the step is captured again before the next replay, so that
        layer's backward reads the stored z instead of recovering it through gamma ~ 0."""
        store = self.trainer.flow_net.store
        guard = store.bn_guard
        if guard is not None and guard.layers:
            before = len(guard.flagged)
            guard.poll()
            if len(guard.flagged) != before:
                torch.cuda.synchronize()
                self._capture()
        if batch_imgs is not None and batch_imgs.data_ptr() != self.batch.data_ptr():
            self.load(batch_imgs)
        if REPLAY_PRIO is None:
            self.graph.replay()
        else:
            # on a stream of its own priority (REPLAY_PRIO: the hipGraphLaunch fault)
            if self._rs is None:
                self._rs = torch.cuda.Stream(priority=REPLAY_PRIO)
            cur = torch.cuda.current_stream()
            self._rs.wait_stream(cur)
            with torch.cuda.stream(self._rs):
                self.graph.replay()
            cur.wait_stream(self._rs)
        store.version += 1
        red = self.trainer.reducer
        if red is not None:
            # the captured step's collectives are not watched inside the capture (an event
            # recorded there would only complete in a replay): bound this replay's instead
            comm = red.comm
            if getattr(comm, "watchdog", None) is not None:
                comm.watch_stream(torch.cuda.current_stream())
                comm.watchdog.check()
        if guard is not None:
            guard.after_update(self.trainer.optimizer.learning_rate)
        return self.loss, self.flows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--height", type=int, default=192)       # train.py:15
    ap.add_argument("--width", type=int, default=640)        # train.py:16
    ap.add_argument("--batch", type=int, default=4)          # train.py:20
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="batches per epoch")
    ap.add_argument("--lr", type=float, default=1e-4)        # train.py:34
    ap.add_argument("--lr-drop-epoch", type=int, default=15)  # train.py:69-70
    ap.add_argument("--pretrained", default=None)
    ap.add_argument("--save-dir", default=None)
    ap.add_argument("--log", default=None, help="JSONL step log")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--kitti", default=None, help="KITTI raw root (train.py:20)")
    ap.add_argument("--nworkers", type=int, default=6)      # train.py:22
    ap.add_argument("--display-dir", default=None, help="PNG flow pictures every 10 batches")
    args = ap.parse_args(argv)

    rank, world, local = init_from_env()
    torch.cuda.set_device(local)
    net = build_flow_net(args.height, args.width, args.pretrained, seed=args.seed)
    if rank == 0:
        net.summary()
    opt = KerasAdam(net.store, learning_rate=args.lr)
    trainer = Trainer(net, opt)
    log = open(args.log, "a") if (args.log and rank == 0) else None
    reader = None
    if args.kitti:
        from .data_reader import AsyncReader, ReaderOpts
        reader = AsyncReader(ReaderOpts(args.kitti, args.batch, args.height, args.width,
                                        args.nworkers, seed=args.seed + rank))
    nbatches = reader.nbatches if reader is not None else args.steps
    step = 0
    for epoch in range(args.epochs):
        if epoch == args.lr_drop_epoch:
            opt.learning_rate = args.lr * 0.1
        t0 = time.time()
        for b in range(nbatches):
            if reader is not None:
                batch = reader.get_batch()
            else:
                batch = torch.from_numpy(synthetic_batch(args.batch, args.height, args.width,
                                                         seed=1234 + step, rank=rank)).cuda()
            loss, flows = trainer.train_step(batch, step)
            lv = float(loss)
            if rank == 0:
                sys.stdout.write("\rbatch %d/%d, loss: %.2e    " % (b + 1, nbatches, lv))
                sys.stdout.flush()
                if log:
                    log.write(json.dumps({"step": step, "loss": lv, "t": time.time() - t0}) + "\n")
                if args.display_dir and (b + 1) % 10 == 0:
                    from .drawing import display_training
                    display_training(batch, flows, args.display_dir, step)
            step += 1
        if rank == 0:
            print("\nEpoch computed in %.3fs" % (time.time() - t0))
            if args.save_dir:
                net.save_weights(os.path.join(args.save_dir, "flow_net_%d" % epoch, "weights"))
    if log:
        log.close()
    if reader is not None:
        reader.close()


if __name__ == "__main__":
    main()
