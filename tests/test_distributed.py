"""CPU, world_size 2 over gloo: the data-parallel pieces of merlin.distributed.

* attach(): rank 0's parameters are broadcast; every rank's .grad is a view of one flat
  buffer that goes to the collective as a single message;
* allreduce_grads(): mean over ranks == the gradient of the mean loss over the
  concatenated batch (equal shard sizes), i.e. the reference's single-learner update;
* advantage moments (count, sum, sum of squares) all-reduced -> normalisation of each
  shard with the concatenated batch's mean / unbiased std (src/ppo.py:125).
"""
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
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from merlin.distributed import DataParallel

        torch.manual_seed(100 + rank)  # different init per rank: attach must unify it
        model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 2))
        dp = DataParallel()
        dp.attach(model)
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        # per-rank shard of a global batch
        g = torch.Generator().manual_seed(7)
        X = torch.randn(world * 16, 6, generator=g)
        Y = torch.randn(world * 16, 2, generator=g)
        xs, ys = X[rank * 16:(rank + 1) * 16], Y[rank * 16:(rank + 1) * 16]
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        dp.zero_grad(opt)
        ((model(xs) - ys) ** 2).mean().backward()
        dp.allreduce_grads()
        grads = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
        # reference: full-batch gradient on rank 0's (broadcast) parameters
        ref_model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 2))
        torch.nn.utils.vector_to_parameters(flat.clone(), ref_model.parameters())
        ((ref_model(X) - Y) ** 2).mean().backward()
        ref_grads = torch.cat([p.grad.reshape(-1) for p in ref_model.parameters()])
        # advantage moments
        adv = torch.from_numpy(np.random.RandomState(rank).randn(1000).astype(np.float32))
        stats = torch.tensor([adv.numel(), adv.double().sum(), (adv.double() ** 2).sum()], dtype=torch.float64)
        dp.allreduce_sum_(stats)
        mean = stats[1] / stats[0]
        std = ((stats[2] - stats[1] * mean) / (stats[0] - 1)).sqrt()
        q.put((rank, flat.numpy(), grads.numpy(), ref_grads.numpy(), float(mean), float(std), dp.world))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_gloo_data_parallel():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, f0, g0, r0, m0, s0, w0), (_, f1, g1, r1, m1, s1, w1) = res
    assert w0 == w1 == 2
    np.testing.assert_array_equal(f0, f1)  # broadcast parameters
    np.testing.assert_allclose(g0, g1, rtol=0, atol=0)  # identical averaged gradients
    np.testing.assert_allclose(g0, r0, rtol=1e-5, atol=1e-7)  # == full-batch gradient
    allv = np.concatenate([np.random.RandomState(r).randn(1000).astype(np.float32) for r in range(2)]).astype(np.float64)
    assert abs(m0 - allv.mean()) < 1e-12 and abs(s0 - allv.std(ddof=1)) < 1e-9
    assert m0 == m1 and s0 == s1
