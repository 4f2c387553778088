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


def selftest(comm, rank: int, world: int, n: int = 4096) -> bool:
    """One small all-reduce checked on the host: every rank contributes rank + 1 (plus a
    position ramp), the sum is known in closed form.  Run once when a data-parallel trainer
    makes its communicator, so an N > 1 RCCL path that cannot sum correctly is caught before
    the first step (it has only ever run at N = 1 on the development boxes)."""
    t = (torch.arange(n, dtype=torch.float32, device="cuda") + (rank + 1)).contiguous()
    comm.allreduce_(t)
    torch.cuda.current_stream().synchronize()
    comm.wait()
    want = torch.arange(n, dtype=torch.float32, device="cuda") * world + world * (world + 1) / 2
    return bool(torch.equal(t, want))


def make_comm(kind: str, rank: int = 0, world: int = 1):
    """"rccl" -> RcclComm(rank, world) on the current device, self-tested (``selftest``) when
    world > 1; if that fails on any rank (the decision is taken jointly over the default
    process group), every rank falls back to torch.distributed's own RCCL (a "nccl" process
    group) with a warning.  "torch" -> TorchComm over the default process group;
    "torch-nccl" -> TorchComm over a new "nccl" group (RCCL through torch)."""
    if kind == "rccl":
        if world <= 1:
            return RcclComm(rank, world)
        import torch.distributed as dist
        comm, ok = None, False
        try:
            comm = RcclComm(rank, world)
            ok = selftest(comm, rank, world)
        except Exception as e:  # noqa: BLE001 -- any failure means: fall back
            import warnings
            warnings.warn("C-ABI RCCL communicator failed on rank %d: %r" % (rank, e))
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)        # control plane (gloo)
        if int(flag) == 1:
            return comm
        import warnings
        warnings.warn("C-ABI RCCL communicator self-test failed: gradients go over "
                      "torch.distributed's nccl (RCCL) backend instead")
        if comm is not None:
            comm.close(abort=True)
        kind = "torch-nccl"
    if kind == "torch":
        return TorchComm()
    if kind == "torch-nccl":
        import torch.distributed as dist
        return TorchComm(dist.new_group(backend="nccl"))
    raise ValueError("comm kind %r (rccl | torch | torch-nccl)" % kind)
