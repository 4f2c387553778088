"""Batch-dimension data parallelism: one process per GPU, gradients summed over RCCL (the C-ABI
communicator of comm.py, over xGMI inside an MI355X node).

The reference is single-process; this is the build-added K14.  Buckets are
contiguous slices of the gradient arena (ordered by backward completion, model.backward_order)
and each is all-reduced (SUM) as soon as every parameter in it has been written by its
backward kernels: the reduction is enqueued on a stream of its own (ops.comm_stream) once that
has waited for the compute stream and the weight-gradient side stream, so RCCL runs after the
producing kernels, the reduction of the finest flow head overlaps the backward of the coarser
levels and the encoder, and a slow peer stalls neither stream.  The compute stream joins the
collective stream at the end of the backward (ops._side_join), before Adam.
The 1/world average is folded into the Adam launch (grad_scale).
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import ops


class GradBucketReducer:
    """comm: a comm.RcclComm / comm.TorchComm (anything with allreduce_(tensor), wait(),
    world); None -> comm.TorchComm over the default process group."""

    def __init__(self, store, bucket_bytes: int = 4 << 20, comm=None):
        self.store = store
        if comm is None:
            from .comm import TorchComm
            comm = TorchComm()
        self.comm = comm
        self.world = comm.world
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
        self._launched: List[bool] = []
        self.launch_log: List[tuple] = []      # (bucket, on the collective stream) per launch

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
        # the wgrad side stream (ops.side_stream): the all-reduce is enqueued on the collective
        # stream once that has waited for both -- during the backward and for the leftovers of
        # finish() alike, so the communicator only ever sees one stream.
        own = _device_tensor(view) and not ops.SINGLE_STREAM
        with (torch.cuda.stream(ops.comm_stream(view, in_backward=in_backward)) if own
              else contextlib.nullcontext()):
            self.comm.allreduce_(view)
        self._launched[bi] = True
        self.launch_log.append((bi, own))

    def begin(self):
        """Arm for one backward pass."""
        self._pending = [len(b) for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self.launch_log = []
        if self.world == 1 and getattr(self.comm, "kind", "") == "torch":
            return            # nothing to reduce, and maybe no process group to reduce over
        ops.set_grad_ready_hook(self._on_grad)

    def finish(self, buffers: Optional[torch.Tensor] = None) -> float:
        """Launch buckets that never completed (unused params) on the collective stream, join
        the reductions (TorchComm: wait on the works; RCCL: stream-ordered, the current stream
        waits for the collective stream here, so only an asynchronous communicator failure is
        checked); returns the grad scale (1/world) for the optimizer.

        ``buffers``: the non-trainable state a step updated on every rank (the BN moving
        statistics in bn_mode "training", ParamStore.buffers) -- replaced by its average over
        the ranks, one more all-reduce on the same stream.  Each rank normalises with its own
        shard's batch statistics (Keras BatchNormalization without synchronisation); the
        moving statistics, identical on every rank before the step, stay identical after it:
        0.99 m + 0.01 mean_r(stat_r)."""
        ops.set_grad_ready_hook(None)
        if self.world == 1 and getattr(self.comm, "kind", "") == "torch":
            return 1.0
        for bi in range(len(self.buckets)):
            if not self._launched[bi]:
                self._launch(bi, in_backward=False)
        if buffers is not None:
            own = _device_tensor(buffers) and not ops.SINGLE_STREAM
            with (torch.cuda.stream(ops.comm_stream(buffers, in_backward=False)) if own
                  else contextlib.nullcontext()):
                self.comm.allreduce_(buffers, average=True)
            self.launch_log.append(("buffers", own))
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            ops.side_join_now()
            # the current stream now waits for every bucket's collective: bound that wait
            # (comm.CommWatchdog aborts the communicator if a peer never joins).  Not while a
            # graph is being captured: an event recorded there completes only in a replay,
            # which GraphedStep watches itself after each replay.
            watch = getattr(self.comm, "watch_stream", None)
            if watch is not None and not torch.cuda.is_current_stream_capturing():
                watch(torch.cuda.current_stream())
        self.comm.wait()
        return 1.0 / self.world


def _device_tensor(t) -> bool:
    """Whether a bucket lives in GPU memory (its all-reduce then gets the collective stream)."""
    return t.is_cuda


def init_from_env(backend: Optional[str] = None):
    """torch.distributed.run environment -> (rank, world, local_rank).  With WORLD_SIZE > 1 the
    default process group is the control plane only -- rendezvous store (which carries the
    RCCL unique id, comm.RcclComm) and barriers -- on gloo unless ``backend`` says otherwise;
    gradients go over the C-ABI RCCL communicator."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = backend or "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local
