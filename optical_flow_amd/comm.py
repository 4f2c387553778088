"""Gradient communicators for the data-parallel train step (SURVEY.md §8 b, §8 e).

``RcclComm`` is the product path: an RCCL communicator behind the C ABI (``of_comm_*`` in
include/oflow.h, csrc/comm.cpp), one per process / GPU.  torch.distributed is plumbing here:
its TCPStore carries rank 0's unique id to the other ranks (the rendezvous of
``torch.distributed.run``), and its (gloo) process group does the bench's barriers; gradient
bytes never go through it.

``TorchComm`` runs the same reducer over a torch.distributed process group -- the gloo
backend on CPU tensors for the multi-process CPU tests, and for two ranks that share one GPU
(an RCCL communicator needs a distinct GPU per rank).
"""
from __future__ import annotations

import ctypes as C
import itertools

import torch

from . import _lib
from ._lib import call

_ids = itertools.count()


def _store():
    import torch.distributed as dist
    if not dist.is_initialized():
        raise RuntimeError("RcclComm with world > 1 needs torch.distributed initialised (its "
                           "TCPStore carries the RCCL unique id)")
    return dist.distributed_c10d._get_default_store()


class RcclComm:
    """One RCCL communicator of ``world`` ranks on the current HIP device.  ``allreduce_``
    sums a float32 CUDA tensor across ranks in place, enqueued on torch's current stream (no
    host wait); ``wait`` only checks the communicator for an asynchronous failure -- ordering
    with later work is stream ordering (the caller's stream waits on the stream it used)."""

    kind = "rccl"

    def __init__(self, rank: int = 0, world: int = 1, store=None, key: str = None):
        lib = _lib.lib()
        self.rank, self.world = rank, world
        nb = lib.of_comm_id_bytes()
        uid = (C.c_char * nb)()
        key = key or "oflow/rccl_id/%d" % next(_ids)
        if rank == 0:
            call("of_comm_get_unique_id", uid)
            if world > 1:
                (store or _store()).set(key, bytes(uid))
        else:
            raw = (store or _store()).get(key)          # blocks until rank 0 has set it
            assert len(raw) == nb, "RCCL unique id: %d bytes, expected %d" % (len(raw), nb)
            C.memmove(uid, raw, nb)
        h = C.c_void_p()
        call("of_comm_init", C.byref(h), uid, world, rank)
        self._h = h
        n, r, d = C.c_int(), C.c_int(), C.c_int()
        call("of_comm_info", h, C.byref(n), C.byref(r), C.byref(d))
        self.device = d.value
        assert (n.value, r.value) == (world, rank)

    def allreduce_(self, t: torch.Tensor):
        if self._h is None:
            raise RuntimeError("RcclComm used after close()")
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise TypeError("RcclComm.allreduce_ takes a contiguous float32 CUDA tensor")
        p = C.c_void_p(t.data_ptr())
        call("of_comm_allreduce_async", self._h, p, p, t.numel(),
             C.c_void_p(torch.cuda.current_stream().cuda_stream))

    def wait(self):
        if self._h is not None:
            call("of_comm_async_error", self._h)

    def close(self, abort: bool = False):
        if self._h is not None:
            h, self._h = self._h, None
            call("of_comm_destroy", h, int(abort))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TorchComm:
    """The reducer's communicator over a torch.distributed process group (gloo in the CPU
    tests): async all_reduce(SUM) per bucket, ``wait`` joins them."""

    kind = "torch"

    def __init__(self, group=None):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self._works = []

    def allreduce_(self, t: torch.Tensor):
        import torch.distributed as dist
        self._works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=True))

    def wait(self):
        for w in self._works:
            w.wait()
        self._works = []

    def close(self, abort: bool = False):
        self._works = []


def make_comm(kind: str, rank: int = 0, world: int = 1):
    """"rccl" -> RcclComm(rank, world) on the current device; "torch" -> TorchComm over the
    default process group."""
    if kind == "rccl":
        return RcclComm(rank, world)
    if kind == "torch":
        return TorchComm()
    raise ValueError("comm kind %r (rccl | torch)" % kind)
