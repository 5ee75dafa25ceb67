"""GPU: data parallelism of merlin.PPO itself (cfg 3's shape), two ranks on one GPU
(torch.distributed, gloo: RCCL needs one GPU per rank) against ONE process over the 2N
concatenated envs.  Rank r owns envs [rN, (r+1)N) seeded 777 + global index, and the action draws
are keyed by the global env index, so each rank's rollout must equal its columns of the single
run bit for bit; the advantages are normalised with the all-reduced global moments
(src/ppo.py:125 over the whole batch) and the rank-averaged gradient of each optimizer step is the
full-minibatch gradient (one step per minibatch, src/ppo.py:153-156) when rank r's minibatch k is
the single run's minibatch k restricted to its envs (the permutations are built that way)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

SMALL = (96, 16, 4, 2)  # N envs per rank, T steps, minibatches, epochs
CFG3 = (4096, 256, 8, 1)  # cfg 3's per-rank shape (4096 envs x 256 steps, 8 minibatches of 131,072)


def _perm(rank_or_none, epoch, shape):
    """Local permutation of rank r (n = N*T), or the single run's (2N*T) made of both ranks'."""
    N, T, MB, _ = shape
    n, m = N * T, N * T // MB
    g = torch.Generator().manual_seed(1000 + epoch)
    local = [torch.randperm(n, generator=g) for _ in range(2)]
    if rank_or_none is not None:
        return local[rank_or_none]

    def to_global(j, r):  # local sample t*N + i -> t*2N + r*N + i
        return (j // N) * 2 * N + r * N + j % N

    parts = []
    for k in range(MB):
        for r in range(2):
            parts.append(to_global(local[r][k * m:(k + 1) * m], r))
    return torch.cat(parts)


def _agent(env, shape, dp=None, rank=None):
    from merlin.ppo import PPO

    _, T, MB, EPOCHS = shape
    torch.manual_seed(5)
    n_envs = env.num_envs
    return PPO(env, batch_size=n_envs * T, minibatch_size=n_envs * T // MB, update_epochs=EPOCHS, ent_coef=0.05,
               device=env.device, dp=dp, perm_fn=lambda n, e: _perm(rank, e, shape))


def _rank_main(rank, port, out_dir, shape):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    import torch.distributed as dist

    from merlin import MerlinVecEnv
    from merlin.distributed import DataParallel

    dist.init_process_group("gloo", rank=rank, world_size=2)
    dev = torch.device("cuda", 0)
    N = shape[0]
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev, env_offset=rank * N)
    agent = _agent(env, shape, DataParallel(), rank)
    lv = agent.collect_rollouts()
    buf = agent.buf
    roll = {k: getattr(buf, k).clone().cpu() for k in ("codes", "actions", "rewards", "dones", "logprobs", "values")}
    stats = agent.update(lv)
    torch.save({"roll": roll, "stats": stats, "adv": agent.last_adv_normalized.clone().cpu(),
                "params": [p.detach().cpu() for p in agent.ac.parameters()], "fast": agent._wstep is not None,
                "windows": agent.last_num_windows},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _two_ranks_vs_one_process(device, tmp_path, shape):
    import torch.multiprocessing as mp

    from merlin import MerlinVecEnv

    N, T, MB, EPOCHS = shape
    mp.start_processes(_rank_main, args=(_free_port(), str(tmp_path), shape), nprocs=2, join=True,
                       start_method="spawn")
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    env = MerlinVecEnv(2 * N, "mediumhard", seed=777, device=device)
    agent = _agent(env, shape)
    lv = agent.collect_rollouts()
    buf = agent.buf
    for r in range(2):  # the rank's rollout is its columns of the single run
        for k, v in res[r]["roll"].items():
            cols = getattr(buf, k).cpu()[:, r * N:(r + 1) * N]
            if k in ("logprobs", "values"):  # the policy GEMMs run at another batch size: fp32 order
                torch.testing.assert_close(v, cols, rtol=1e-5, atol=1e-5)
            else:  # observations, actions, rewards, dones: bit for bit
                assert torch.equal(v, cols), (r, k)
    stats = agent.update(lv)
    # global-moment normalisation: each rank's advantages == the single run's columns
    for r in range(2):
        torch.testing.assert_close(res[r]["adv"], agent.last_adv_normalized.cpu()[:, r * N:(r + 1) * N],
                                   rtol=1e-5, atol=1e-5)
    for k in stats:
        dp_val = 0.5 * (res[0]["stats"][k] + res[1]["stats"][k]) if k != "gradnorm" else res[0]["stats"][k]
        # clipfrac counts samples with |ratio - 1| > clip: a ratio within fp32 noise of the boundary flips with the
        # summation order (4 samples per minibatch, or 1 in 10^4 at cfg 3's 262,144-sample minibatches)
        tol = max(4.0 / (2 * N * T // MB), 1e-4) if k == "clipfrac" else 1e-4 * max(1.0, abs(stats[k]))
        assert abs(dp_val - stats[k]) <= tol, (k, dp_val, stats[k])
    # replicated parameters: both ranks identical; vs the single run within the Adam-step bound of
    # test_gpu_windows.py (fp32 summation order differs: per-rank dedup groups, all-reduced sums)
    for a, b in zip(res[0]["params"], res[1]["params"]):
        assert torch.equal(a, b)
    ds = [(a - b.detach().cpu()).abs().flatten() for a, b in zip(res[0]["params"], agent.ac.parameters())]
    steps = EPOCHS * MB
    for d in ds:
        assert d.max().item() <= 2 * 3e-4 * steps
    assert (torch.cat(ds) > 5e-5).float().mean().item() < 0.05
    return res, agent


def test_two_rank_ppo_equals_one_process_over_concatenated_envs(device, tmp_path):
    _two_ranks_vs_one_process(device, tmp_path, SMALL)


def test_two_rank_ppo_cfg3_per_rank_shape(device, tmp_path):
    """cfg 3's per-rank work (4096 envs x 256 steps, 8 minibatches of 131,072: the benched path with windows,
    distinct-frame grouping, the fast step, per-rank plans) under a process group, against one process over the
    8,192 concatenated envs."""
    res, agent = _two_ranks_vs_one_process(device, tmp_path, CFG3)
    assert all(r["fast"] for r in res) and agent._wstep is not None  # the benched step ran on both sides
    assert all(r["windows"] and r["windows"] > 1000 for r in res)
