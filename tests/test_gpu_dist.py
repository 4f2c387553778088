"""The data-parallel train step on the GPU path: two ranks share the one GPU of the box (gloo
carries the all-reduce of CUDA tensors; the N>1 bench runs the same reducer over RCCL).  The
bucket all-reduces are launched during the backward, ordered after the weight-gradient side
stream (ops.side_stream).  The gradient of two 1-pair shards, summed by the all-reduce and
scaled by 1/world, must equal that of a single process on the 2-pair batch (P10)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

H, W = 64, 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _step(batch_np, rank=None, world=1):
    from optical_flow_amd.model import FlowNet
    from optical_flow_amd.params import flow_net_spec, init_params, perturb_params
    from optical_flow_amd.train import KerasAdam, Trainer
    vals = perturb_params(init_params(flow_net_spec(), 0), 1)
    net = FlowNet(H, W, values=vals)
    trainer = Trainer(net, KerasAdam(net.store, learning_rate=1e-3),
                      data_parallel=world > 1)
    x = torch.from_numpy(batch_np if rank is None else batch_np[rank:rank + 1]).cuda()
    trainer.train_step(x, 0)
    torch.cuda.synchronize()
    return net.store.grad_arena.cpu().numpy() / world


def _worker(rank, world, port, batch_np, q):
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        q.put((rank, _step(batch_np, rank, world)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_data_parallel_step_matches_single_process():
    from optical_flow_amd.data import synthetic_batch
    batch = synthetic_batch(2, H, W, seed=23)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    ref = _step(batch)
    assert np.isfinite(ref).all() and np.abs(ref).max() > 0
    np.testing.assert_array_equal(res[0], res[1])          # replicas hold the same average
    # equal-shard average == global-batch gradient (P10), up to fp32 summation order (split-K
    # plans depend on the batch size; measured ~1e-7)
    err = np.linalg.norm(res[0] - ref) / np.linalg.norm(ref)
    print("DP vs single-process gradient rel_l2 %.2e" % err)
    assert err < 1e-4, err
