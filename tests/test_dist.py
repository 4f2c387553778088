"""Data-parallel path on CPU with the gloo backend, world size 2 (the N>1 bench runs the same
code over RCCL): gradient-bucket reducer semantics, and equal-shard gradient averaging equals
the global-batch gradient under the reference loss (P10)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _reducer_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from optical_flow_amd import ops
        from optical_flow_amd.dist import GradBucketReducer
        from optical_flow_amd.model import ParamStore, backward_order
        from optical_flow_amd.params import flow_net_spec
        st = ParamStore(flow_net_spec(), device="cpu", order=backward_order())
        st.grad_arena.copy_(torch.arange(st.numel, dtype=torch.float32) * (rank + 1))
        red = GradBucketReducer(st, bucket_bytes=2 << 20)
        red.begin()
        launched = []
        for name in st.arena_order:                 # backward completion order
            ops._grad_ready(st.params[name])
            launched.append(sum(red._launched))
        scale = red.finish()
        ok = torch.equal(st.grad_arena, torch.arange(st.numel, dtype=torch.float32) * 3)
        # buckets launch progressively during the backward, not all at the end
        q.put((rank, ok, scale, len(red.buckets), launched[len(launched) // 2]))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None, None, None))


def test_grad_bucket_reducer_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok, scale, nb, mid in res:
        assert ok is True, ok
        assert scale == 0.5
        assert nb >= 5
        assert 0 < mid < nb


def _oracle_dp_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from oracle import ref_flow as R
        from optical_flow_amd.data import synthetic_batch
        from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params
        torch.set_num_threads(2)
        vals = init_params(flow_net_spec(), 0)
        full = synthetic_batch(2, 32, 64, seed=5)
        p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
        _, _, g = R.train_step(torch.tensor(full[rank:rank + 1], dtype=torch.float64), p,
                               list(encoder_blocks()), None)
        names = sorted(g)
        flat = torch.cat([g[k].flatten() for k in names])
        dist.all_reduce(flat)
        flat /= world
        q.put((rank, flat.numpy()))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_data_parallel_average_equals_global_batch():
    from oracle import ref_flow as R
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_oracle_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert not isinstance(res[0], str), res[0]
    vals = init_params(flow_net_spec(), 0)
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    _, _, g = R.train_step(torch.tensor(synthetic_batch(2, 32, 64, seed=5), dtype=torch.float64),
                           p, list(encoder_blocks()), None)
    ref = torch.cat([g[k].flatten() for k in sorted(g)]).numpy()
    np.testing.assert_allclose(res[0], ref, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(res[1], ref, rtol=1e-9, atol=1e-12)


def test_bucket_allreduce_on_collective_stream(monkeypatch):
    """Every bucket's all-reduce is enqueued on the collective stream (ops.comm_stream:
    ordered after the compute and weight-gradient side streams), never on the side stream or
    the current stream -- during the backward and for the leftovers of finish() alike (one
    communicator, one stream: RCCL requires a communicator's operations in the same order on
    every rank) --, in backward-completion (arena) order, each bucket exactly once; the
    buffers' average goes on the same stream last.  (Streams stubbed: CPU.)"""
    import contextlib
    from optical_flow_amd import dist as D
    from optical_flow_amd import ops
    from optical_flow_amd.model import ParamStore, backward_order
    from optical_flow_amd.params import flow_net_spec
    calls = []

    class FakeComm:
        kind, world = "fake", 2

        def allreduce_(self, t, average=False):
            calls.append(("allreduce", t.data_ptr(), t.numel(), average))

        def wait(self):
            calls.append(("wait",))

    st = ParamStore(flow_net_spec(), device="cpu", order=backward_order())
    red = D.GradBucketReducer(st, bucket_bytes=2 << 20, comm=FakeComm())
    monkeypatch.setattr(D, "_device_tensor", lambda t: True)
    monkeypatch.setattr(ops, "comm_stream", lambda *t, in_backward=True: calls.append(
        ("comm_stream", t[0].data_ptr(), in_backward)) or "S")
    monkeypatch.setattr(ops, "side_stream", lambda *t: (_ for _ in ()).throw(AssertionError("side")))
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    red.begin()
    names = st.arena_order
    held = names[-1]                             # one parameter never reports: a leftover
    for name in names[:-1]:
        ops._grad_ready(st.params[name])
    assert red.finish(buffers=st.buffers) == 0.5
    nb = len(red.buckets)
    assert [b for b, _ in red.launch_log] == list(range(nb)) + ["buffers"]
    assert all(own for _, own in red.launch_log)
    ar = [c for c in calls if c[0] == "allreduce"]
    cs = [c for c in calls if c[0] == "comm_stream"]
    assert len(ar) == nb + 1 and len(cs) == nb + 1
    for (lo, hi), c in zip(red.ranges, ar):
        assert c[1] == st.grad_arena[lo:hi].data_ptr() and c[2] == hi - lo and not c[3]
    assert ar[-1] == ("allreduce", st.buffers.data_ptr(), st.buffers.numel(), True)
    # every collective-stream fork precedes its all-reduce; the backward's forks arm the
    # end-of-backward join, the leftover's and the buffers' (after the backward) do not
    for i in range(nb + 1):
        k = calls.index(cs[i])
        assert calls[k + 1] == ar[i]
    assert [c[2] for c in cs] == [True] * (nb - 1) + [False, False]
    assert held in red.buckets[-1]


def _bn_stats_worker(rank, world, port, q):
    """bn_mode "training" under data parallelism: each rank's oracle step updates the moving
    statistics with its own shard's batch statistics; the reducer's buffer average leaves
    both replicas with the same statistics, 0.99 m + 0.01 mean over ranks of the per-rank
    statistics."""
    try:
        _init(rank, world, port)
        from oracle import ref_flow as R
        from optical_flow_amd.data import synthetic_batch
        from optical_flow_amd.dist import GradBucketReducer
        from optical_flow_amd.model import ParamStore, backward_order
        from optical_flow_amd.params import encoder_blocks, flow_net_spec, init_params
        torch.set_num_threads(2)
        vals = init_params(flow_net_spec(), 3)
        full = synthetic_batch(2, 32, 64, seed=8)
        p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
        R.set_bn_mode("training")
        R.train_step(torch.tensor(full[rank:rank + 1], dtype=torch.float64), p,
                     list(encoder_blocks()), None)
        st = ParamStore(flow_net_spec(), values=vals, device="cpu", order=backward_order())
        mine = {n: p[n].float() for n in st.buf_offsets}
        with torch.no_grad():
            for n, v in mine.items():
                st.params[n].copy_(v)
        red = GradBucketReducer(st, bucket_bytes=2 << 20)
        red.begin()
        red.finish(buffers=st.buffers)
        q.put((rank, {n: st.params[n].clone().numpy() for n in st.buf_offsets},
               {n: v.numpy() for n, v in mine.items()}))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


def test_bn_training_moving_statistics_replicas_equal():
    res = {r: (a, b) for r, a, b in _run2(_bn_stats_worker)}
    assert not isinstance(res[0][0], str), res[0][0]
    assert not isinstance(res[1][0], str), res[1][0]
    (s0, own0), (s1, own1) = res[0], res[1]
    assert set(s0) and set(s0) == set(s1)
    moved = 0
    for n in s0:
        np.testing.assert_array_equal(s0[n], s1[n])              # replicas identical
        np.testing.assert_allclose(s0[n], (own0[n] + own1[n]) / 2, rtol=1e-6, atol=1e-7)
        moved += int(not np.array_equal(own0[n], own1[n]))
    assert moved > len(s0) // 2          # the per-rank updates did differ before the average


# ---------------------------------------------------------------------------------------------
# N > 1 communicator set-up without hardware: the joint fallback vote and the
# deadlines, with the RCCL communicator replaced by fakes (an RCCL communicator needs one GPU
# per rank; these paths are host logic).
class _FakeRccl:
    kind = "rccl"

    def __init__(self, rank, world, timeout=None, **kw):
        if rank == 1:
            raise RuntimeError("simulated of_comm_init failure on rank 1")
        self.rank, self.world, self.closed = rank, world, None

    def close(self, abort=False):
        self.closed = abort


def _vote_worker(rank, world, port, q, mode):
    try:
        _init(rank, world, port)
        from optical_flow_amd import comm as CM
        CM.RcclComm = _FakeRccl
        CM.selftest = lambda c, r, w: True
        if mode == "fallback":
            c = CM.make_comm("rccl", rank, world, fallback="torch", timeout=30)
            t = torch.full((4,), float(rank + 1))
            c.allreduce_(t)
            c.wait()
            q.put((rank, c.kind, float(t[0])))
        else:                              # "timeout": rank 1 never votes
            if rank == 0:
                try:
                    CM.make_comm("rccl", rank, world, fallback="torch", timeout=2)
                    q.put((rank, "no error", None))
                except CM.CommError as e:
                    q.put((rank, "CommError", str(e)[:80]))
            else:
                q.put((rank, "skipped", None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


def _run2(target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, 2, port, q) + args) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return res


def test_make_comm_joint_fallback():
    """comm.make_comm's vote (through the rendezvous store, not a collective): the RCCL
    communicator fails on rank 1 only, and BOTH ranks must end on the same fallback -- whose
    all-reduce then works (1 + 2 = 3)."""
    res = _run2(_vote_worker, "fallback")
    assert res == [(0, "torch", 3.0), (1, "torch", 3.0)], res


def test_make_comm_vote_deadline():
    """A rank that never reaches the vote makes the other one raise CommError after the
    deadline instead of blocking forever."""
    res = _run2(_vote_worker, "timeout")
    assert res[0][:2] == (0, "CommError"), res
    assert res[1][:2] == (1, "skipped"), res


def test_comm_watchdog():
    """comm.CommWatchdog: a completion predicate that never turns true expires after the
    timeout (on_expire is called once, check() raises CommError in the caller's thread); one
    that completes is dropped; an asynchronous communicator error fails at once."""
    import time
    from optical_flow_amd.comm import CommError, CommWatchdog
    seen = []
    w = CommWatchdog(0.3, seen.append, poll_s=0.005)
    w.watch(lambda: True)
    t0 = time.monotonic()
    while w.pending() and time.monotonic() - t0 < 5:
        time.sleep(0.01)
    assert w.pending() == 0 and w.failed is None
    w.check()
    w.watch(lambda: False)
    while w.failed is None and time.monotonic() - t0 < 5:
        time.sleep(0.01)
    assert len(seen) == 1 and "did not complete" in seen[0]
    with pytest.raises(CommError):
        w.check()
    w.close()
    seen2 = []
    w2 = CommWatchdog(60, seen2.append, poll_s=0.005, error_probe=lambda: "RCCL failed: x")
    w2.watch(lambda: False)
    t0 = time.monotonic()
    while w2.failed is None and time.monotonic() - t0 < 5:
        time.sleep(0.01)
    assert seen2 == ["RCCL failed: x"]
    w2.close()


def test_vote_single_process_store():
    """comm.vote over a store: all ok -> True, one not ok -> False (a HashStore, world 1 and
    a pre-set second vote)."""
    from optical_flow_amd.comm import vote
    st = dist.HashStore()
    assert vote(st, "t1", 0, 1, True, timeout=2) is True
    st.set("t2/1", b"0")
    assert vote(st, "t2", 0, 2, True, timeout=2) is False
