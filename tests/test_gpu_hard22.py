"""GPU: BASELINE cfg 4 -- hard difficulty on 22x22 grids (src/custom_envs/hard_env.py:11-97), 4096 envs --
through the full PPO loop, as tests/test_gpu_fullsize.py does for cfg 2:

  * the rollout of merlin.PPO (act -> env step -> auto-reset, look-ahead map refills on the side stream)
    replays bit-exact through the C oracle (oracle/merlin_oracle.c, the restatement of hard_env.py's
    _gen_grid / minigrid step / view) fed the rollout's own actions: observation codes, rewards and
    done flags of all 4096 envs;
  * the next rollout, replayed from the captured HIP graph, equals an eager env continuing the same
    PCG64 streams;
  * one update through the benched path (windows, distinct frames, x6 fc1, fused loss, clip + Adam)
    against the per-frame lookup path on the same rollout (tolerances of test_gpu_windows.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, T, MAX_STEPS = 4096, 64, 40  # max_steps 40 < T: every env ends episodes inside the rollout


def _unpack(codes):
    w = codes.cpu().numpy().astype(np.uint32)
    nib = (w[..., :, None] >> (4 * np.arange(8, dtype=np.uint32))) & 0xF
    return nib.reshape(*w.shape[:-1], 64)[..., :49]


def test_cfg4_rollout_vs_oracle_and_graph_replay(oracle, device):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    env = MerlinVecEnv(N, "hard", size=22, seed=777, device=device, max_steps=MAX_STEPS)
    torch.manual_seed(0)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=1, ent_coef=0.05, device=device)
    buf = agent.buf
    agent.collect_rollouts()  # eager (the graph is captured after it)
    acts = buf.actions.cpu().numpy()
    ocodes, orew, oterm, otrunc, _ = oracle.batch_rollout(np.arange(777, 777 + N, dtype=np.uint64), acts,
                                                          size=22, difficulty="hard", max_steps=MAX_STEPS)
    assert (_unpack(buf.codes) == ocodes).all()
    assert (buf.rewards.cpu().numpy() == orew).all()
    assert (buf.dones.cpu().numpy() == np.maximum(oterm, otrunc)).all()
    assert otrunc.sum() >= N  # every env truncated at least once
    # second rollout from the captured graph == an eager env continuing the same streams
    mirror = MerlinVecEnv(N, "hard", size=22, seed=777, device=device, max_steps=MAX_STEPS)
    scratch = torch.zeros((N, 8), dtype=torch.int32, device=device)
    mirror.reset(out=scratch)
    for t in range(T):  # replay rollout 1 on the mirror (eager)
        mirror.step_into(buf.actions[t].contiguous(), scratch, torch.empty(N, device=device), None, None,
                         torch.empty(N, device=device))
    agent.update(buf.last_value)
    agent.collect_rollouts()
    assert agent._graph is not None
    codes = torch.zeros_like(buf.codes)
    rew, done = torch.zeros_like(buf.rewards), torch.zeros_like(buf.dones)
    mirror.reset(out=codes[0])
    for t in range(T):
        mirror.step_into(buf.actions[t].contiguous(), codes[t + 1], rew[t], None, None, done[t])
    assert torch.equal(codes, buf.codes)
    assert torch.equal(rew, buf.rewards) and torch.equal(done, buf.dones)
    env.errors()
    mirror.errors()


def test_cfg4_window_update_matches_lookup_path(device):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    res = []
    for windows in (True, False):
        env = MerlinVecEnv(N, "hard", size=22, seed=777, device=device)
        torch.manual_seed(3)
        g = torch.Generator(device=device)
        g.manual_seed(11)
        agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=1, ent_coef=0.05,
                    device=device, windows=windows,
                    perm_fn=lambda n, e: torch.randperm(n, device=device, generator=g))
        torch.manual_seed(4)
        stats = agent.update(agent.collect_rollouts())
        res.append((stats, [p.detach().clone() for p in agent.ac.parameters()], agent.last_num_windows,
                    agent.buf.codes.clone()))
        env.close()
    (s1, p1, nw, c1), (s2, p2, none, c2) = res
    assert torch.equal(c1, c2)  # same rollout (counter-based action draws, same seeds)
    assert none is None and nw > 0
    for k in s1:
        tol = 4.0 / (N * T // 4) if k == "clipfrac" else 1e-4 * max(1.0, abs(s2[k]))
        assert abs(s1[k] - s2[k]) <= tol, (k, s1[k], s2[k])
    ds = [(a - b).abs().flatten() for a, b in zip(p1, p2)]
    for d in ds:
        assert d.max().item() <= 2 * 3e-4 * 4
    assert (torch.cat(ds) > 5e-5).float().mean().item() < 0.05
