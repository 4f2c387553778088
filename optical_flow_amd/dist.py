"""Batch-dimension data parallelism: one process per GPU, gradients all-reduced with
torch.distributed (backend "nccl" = RCCL on ROCm, over xGMI inside an MI355X node).

The reference is single-process; this is the build-added K14.  Buckets are
contiguous slices of the gradient arena (ordered by backward completion, model.backward_order)
and each is all-reduced (SUM) as soon as every parameter in it has been written by its
backward kernel -- RCCL runs on its own stream, ordered after the producing kernels, so the
reduction of the finest flow head overlaps the backward of the coarser levels and the encoder.
The 1/world average is folded into the Adam launch (grad_scale).
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import ops


class GradBucketReducer:
    def __init__(self, store, bucket_bytes: int = 4 << 20, group=None):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # bucket = contiguous arena range covering whole parameters
        self.buckets: List[List[str]] = []
        cur, cur_bytes = [], 0
        for name in store.arena_order:
            size = store.spec[name].size * 4
            if cur and cur_bytes + size > bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(name)
            cur_bytes += size
        if cur:
            self.buckets.append(cur)
        self.bucket_of: Dict[int, int] = {}
        self.ranges = []
        for bi, names in enumerate(self.buckets):
            lo = store.offsets[names[0]]
            last = names[-1]
            hi = store.offsets[last] + (store.spec[last].size + 3) // 4 * 4
            self.ranges.append((lo, hi))
            for n in names:
                self.bucket_of[id(store.params[n])] = bi
        self._pending: List[int] = []
        self._works = []
        self._launched: List[bool] = []

    # -- called by ops after a parameter's gradient kernels are enqueued -----------------
    def _on_grad(self, param):
        bi = self.bucket_of.get(id(param))
        if bi is None or self._launched[bi]:
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi, in_backward=True):
        lo, hi = self.ranges[bi]
        view = self.store.grad_arena[lo:hi]
        # A bucket's gradients are written on the current stream (BN / bias reductions) and on
        # the wgrad side stream (ops.side_stream): during the backward the all-reduce is
        # enqueued on the side stream once it has waited for the current one, so RCCL is
        # ordered after both without stalling the input-gradient chain.
        side = in_backward and view.is_cuda and ops.SIDE_STREAM_WGRAD
        with torch.cuda.stream(ops.side_stream()) if side else contextlib.nullcontext():
            self._works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))
        self._launched[bi] = True

    def begin(self):
        """Arm for one backward pass."""
        self._pending = [len(b) for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._works = []
        ops.set_grad_ready_hook(self._on_grad if self.world > 1 else None)

    def finish(self) -> float:
        """Launch buckets that never completed (unused params), make the current stream wait
        for every reduction; returns the grad scale (1/world) for the optimizer."""
        ops.set_grad_ready_hook(None)
        if self.world > 1:
            for bi in range(len(self.buckets)):
                if not self._launched[bi]:
                    self._launch(bi, in_backward=False)
            for w in self._works:
                w.wait()
        self._works = []
        return 1.0 / self.world


def init_from_env(backend: Optional[str] = None):
    """torch.distributed.run environment -> (rank, world, local_rank); initialises the
    process group when WORLD_SIZE > 1."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local
