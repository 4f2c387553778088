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
import datetime
import itertools
import os
import threading
import time

import torch

from . import _lib
from ._lib import OF_OK, OflowTimeout, call

_ids = itertools.count()
_votes = itertools.count()

# Deadline (seconds) for every step of the N > 1 communicator that waits on peers: the probe
# exchange and the RCCL rendezvous at init, the self-test all-reduce, and each step's bucket
# all-reduces (CommWatchdog).  A peer that never arrives then ends in an error on every rank
# instead of a hang.  OFLOW_COMM_TIMEOUT overrides.
COMM_TIMEOUT_S = float(os.environ.get("OFLOW_COMM_TIMEOUT", "300"))


class CommError(RuntimeError):
    """The gradient communicator failed or timed out (SURVEY.md §5 failure detection)."""


def _store_wait(store, keys, timeout):
    try:
        store.wait(list(keys), datetime.timedelta(seconds=timeout))
    except Exception as e:  # noqa: BLE001 -- the store raises its own timeout types
        raise CommError("rendezvous store: %d key(s) %s not set within %.0f s (a peer is "
                        "missing or failed before reaching this point): %r" % (
                            len(keys), list(keys)[:3], timeout, e)) from e


def vote(store, tag: str, rank: int, world: int, ok: bool, timeout: float = None) -> bool:
    """All ranks' verdicts through the rendezvous store (no collective on any process group,
    so it works whatever backend the default group has): True iff every rank voted ok.  A
    rank that never votes makes every other rank raise CommError after ``timeout``."""
    timeout = COMM_TIMEOUT_S if timeout is None else timeout
    store.set("%s/%d" % (tag, rank), b"1" if ok else b"0")
    keys = ["%s/%d" % (tag, r) for r in range(world)]
    _store_wait(store, keys, timeout)
    return all(bytes(store.get(k)) == b"1" for k in keys)


class CommWatchdog:
    """Bounds the waits a data-parallel step cannot bound itself: each step's
    collectives are stream-ordered, so nothing on the host waits for them -- a peer that never
    joins would hang the next synchronize.  ``watch(done)`` registers a completion predicate
    (an event recorded after the step's last collective); a daemon thread polls it, and the
    communicator's asynchronous error state, and after ``timeout`` seconds calls
    ``on_expire(reason)`` (RcclComm: abort the communicator, which makes its in-flight kernels
    return) and remembers the reason; ``check()`` raises CommError with it in the caller's
    thread (GradBucketReducer.finish, once per step)."""

    def __init__(self, timeout: float, on_expire, poll_s: float = 0.01, error_probe=None):
        self.timeout = timeout
        self.on_expire = on_expire
        self.error_probe = error_probe
        self.poll_s = poll_s
        self.failed = None
        self._q = []
        self._cv = threading.Condition()
        self._stop = False
        self._t = threading.Thread(target=self._run, name="oflow-comm-watchdog", daemon=True)
        self._t.start()

    def watch(self, done):
        with self._cv:
            self._q.append((done, time.monotonic() + self.timeout))
            self._cv.notify()

    def pending(self) -> int:
        with self._cv:
            return len(self._q)

    def check(self):
        if self.failed is not None:
            raise CommError(self.failed)

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._t.join(timeout=5)

    def _fail(self, reason):
        with self._cv:
            if self.failed is not None:
                return
            self.failed = reason
            self._q.clear()
        try:
            self.on_expire(reason)
        except Exception:  # noqa: BLE001 -- the reason is kept for check()
            pass

    def _run(self):
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if self._stop:
                    return
                done, deadline = self._q[0]
            try:
                finished = done()
            except Exception as e:  # noqa: BLE001
                self._fail("collective completion check raised %r" % (e,))
                continue
            if finished:
                with self._cv:
                    if self._q and self._q[0][0] is done:
                        self._q.pop(0)
                continue
            err = self.error_probe() if self.error_probe is not None else None
            if err:
                self._fail(err)
            elif time.monotonic() > deadline:
                self._fail("a step's gradient all-reduce did not complete within %.0f s (a "
                           "peer stopped joining the collectives); communicator aborted" %
                           self.timeout)
            else:
                time.sleep(self.poll_s)


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

    def __init__(self, rank: int = 0, world: int = 1, store=None, key: str = None,
                 timeout: float = None):
        lib = _lib.lib()
        self.rank, self.world = rank, world
        self.timeout = COMM_TIMEOUT_S if timeout is None else timeout
        self._h = None
        self.watchdog = None
        nb = lib.of_comm_id_bytes()
        uid = (C.c_char * nb)()
        key = key or "oflow/rccl_id/%d" % next(_ids)
        if world > 1:
            store = store or _store()
            # every rank checks that it can make a communicator at all (librccl, a device)
            # and the ranks agree on it through the store BEFORE any of them enters the RCCL
            # rendezvous, which would otherwise wait for a rank that already gave up
            ok = lib.of_comm_probe() == OF_OK
            why = "" if ok else lib.of_last_error().decode(errors="replace")
            if not vote(store, key + "/probe", rank, world, ok, self.timeout):
                raise CommError("C-ABI RCCL communicator unavailable on at least one rank%s" % (
                    (" (this rank: %s)" % why) if why else ""))
        if rank == 0:
            call("of_comm_get_unique_id", uid)
            if world > 1:
                store.set(key, bytes(uid))
        else:
            _store_wait(store, [key], self.timeout)
            raw = store.get(key)
            assert len(raw) == nb, "RCCL unique id: %d bytes, expected %d" % (len(raw), nb)
            C.memmove(uid, raw, nb)
        h = C.c_void_p()
        try:
            call("of_comm_init_timeout", C.byref(h), uid, world, rank,
                 self.timeout if world > 1 else 0.0)
        except OflowTimeout as e:
            raise CommError(str(e)) from e
        self._h = h
        n, r, d = C.c_int(), C.c_int(), C.c_int()
        call("of_comm_info", h, C.byref(n), C.byref(r), C.byref(d))
        self.device = d.value
        assert (n.value, r.value) == (world, rank)
        self._lock = threading.Lock()
        if world > 1:
            self.watchdog = CommWatchdog(self.timeout, self._expire, error_probe=self._probe)

    def _probe(self):
        """The communicator's asynchronous error, as text (None while healthy)."""
        with self._lock:
            if self._h is None:
                return None
            st = _lib.lib().of_comm_async_error(self._h)
            if st == OF_OK:
                return None
            return "RCCL communicator failed: " + _lib.lib().of_last_error().decode(
                errors="replace")

    def _expire(self, reason):
        """Watchdog thread: abort the communicator's in-flight collectives (their kernels
        return) but keep the handle -- the owner thread may be inside allreduce_ / wait with
        it; those fail cleanly on an aborted handle, and close() frees it later."""
        with self._lock:
            if self._h is not None:
                _lib.lib().of_comm_abort(self._h)

    def watch_stream(self, stream):
        """Bound the collectives enqueued so far on ``stream`` (an event recorded there; the
        watchdog aborts the communicator if it is not reached within the timeout)."""
        if self.watchdog is None:
            return
        ev = torch.cuda.Event()
        ev.record(stream)
        self.watchdog.watch(ev.query)

    def allreduce_(self, t: torch.Tensor, average: bool = False):
        """In place: the sum over ranks (average: the mean, OF_REDUCE_AVG)."""
        if self.watchdog is not None:
            self.watchdog.check()
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise TypeError("RcclComm.allreduce_ takes a contiguous float32 CUDA tensor")
        p = C.c_void_p(t.data_ptr())
        with self._lock:                 # the watchdog's abort never races this call
            if self._h is None:
                raise RuntimeError("RcclComm used after close()")
            call("of_comm_allreduce_ex_async", self._h, p, p, t.numel(),
                 _lib.OF_REDUCE_AVG if average else _lib.OF_REDUCE_SUM,
                 C.c_void_p(torch.cuda.current_stream().cuda_stream))

    def wait(self):
        if self.watchdog is not None:
            self.watchdog.check()
        with self._lock:
            if self._h is not None:
                call("of_comm_async_error", self._h)

    def close(self, abort: bool = False):
        lock = getattr(self, "_lock", None)
        with lock if lock is not None else _nolock():
            h, self._h = self._h, None
        if self.watchdog is not None and threading.current_thread() is not self.watchdog._t:
            self.watchdog.close()
        if h is not None:
            call("of_comm_destroy", h, int(abort))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _nolock:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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

    def allreduce_(self, t: torch.Tensor, average: bool = False):
        """average: the mean over ranks (gloo has no AVG: SUM, divided by the world size when
        the work is joined in wait())."""
        import torch.distributed as dist
        w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._works.append((w, t if average else None))

    def wait(self):
        for w, avg in self._works:
            w.wait()
            if avg is not None:
                avg.div_(self.world)
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
    ev = torch.cuda.Event()
    ev.record()
    deadline = time.monotonic() + getattr(comm, "timeout", COMM_TIMEOUT_S)
    while not ev.query():          # bounded: a hung peer must not hang this rank's init
        if time.monotonic() > deadline:
            comm.close(abort=True)
            raise CommError("RCCL self-test all-reduce did not complete within %.0f s" %
                            getattr(comm, "timeout", COMM_TIMEOUT_S))
        time.sleep(0.001)
    comm.wait()
    want = torch.arange(n, dtype=torch.float32, device="cuda") * world + world * (world + 1) / 2
    return bool(torch.equal(t, want))


def make_comm(kind: str, rank: int = 0, world: int = 1, fallback: str = "torch-nccl",
              timeout: float = None):
    """"rccl" -> RcclComm(rank, world) on the current device, self-tested (``selftest``) when
    world > 1; if making or testing it fails on any rank, every rank falls back together to
    ``fallback`` (default torch.distributed's own RCCL, a "nccl" process group) with a warning.
    The decision is a ``vote`` through the rendezvous store, not a collective on the default
    process group (whatever its backend), and every wait on a peer has a deadline (``timeout``,
    default COMM_TIMEOUT_S): a rank that dies or hangs before voting makes the others raise
    CommError instead of hanging.  "torch" -> TorchComm over the default process group;
    "torch-nccl" -> TorchComm over a new "nccl" group (RCCL through torch)."""
    if kind == "rccl":
        if world <= 1:
            return RcclComm(rank, world)
        import warnings
        timeout = COMM_TIMEOUT_S if timeout is None else timeout
        tag = "oflow/make_comm/%d" % next(_votes)
        comm, ok = None, False
        try:
            comm = RcclComm(rank, world, timeout=timeout)
            ok = selftest(comm, rank, world)
        except Exception as e:  # noqa: BLE001 -- any failure means: fall back
            warnings.warn("C-ABI RCCL communicator failed on rank %d: %r" % (rank, e))
        if vote(_store(), tag, rank, world, ok, timeout):
            return comm
        warnings.warn("C-ABI RCCL communicator failed its set-up or self-test on at least one "
                      "rank: gradients go over %s instead (all ranks)" % fallback)
        if comm is not None:
            comm.close(abort=True)
        kind = fallback
    if kind == "torch":
        return TorchComm()
    if kind == "torch-nccl":
        import torch.distributed as dist
        return TorchComm(dist.new_group(backend="nccl"))
    raise ValueError("comm kind %r (rccl | torch | torch-nccl)" % kind)
