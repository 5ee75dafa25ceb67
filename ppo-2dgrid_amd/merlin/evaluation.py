"""Batched deterministic evaluation and the checkpoint sweep.

``evaluate_policy``  ppo/ppo_train.py:43-69 of the reference: episode ep is reset with
                     ``seed = base_seed + ep`` and run to termination/truncation with the argmax
                     policy.  Here all episodes run at once in one ``MerlinVecEnv`` (env ep seeded
                     base_seed + ep: the same maps), one batched deterministic forward per step, no
                     auto-reset; an env's result is frozen at its first done.  Episode returns are
                     the env's f64 accumulator (the reference sums Python floats), not a sum of the
                     f32 reward buffer.
``evaluate_seeds``   the same for an arbitrary list of seeds (src/sweep_checkpoints.py:52-70
                     evaluate_model: one episode per seed, returns the mean reward and steps).
``sweep_checkpoints`` src/sweep_checkpoints.py:72-100: every ``*.pth`` of a directory on the fixed
                     seeds 200000 + i, ranked by mean reward; checkpoints load through
                     merlin.checkpoints.load_policy (legacy-key remap included).
``evaluate_zero_shot`` src/distribution_over_tasks.py:71-120 for many seeds at once: the
                     deterministic episode's reward and length, and its PPO-style loss -- GAE
                     (gamma .995, lambda .95) over the episode with the value after the last step
                     masked out, advantages normalised over the episode (zeros for a 1-step
                     episode), returns = values + advantages, then -mean(logp) + 0.5 * mean((v -
                     return)^2) with the episode's observations re-evaluated.
"""
from __future__ import annotations

import glob
import os

import torch

from .envs import MerlinVecEnv

SWEEP_SEED_BASE = 200000  # src/sweep_checkpoints.py:79


@torch.no_grad()
def evaluate_seeds(ac, seeds, difficulty: str = "mediumhard", size: int = 16, device="cuda",
                   max_steps: int | None = None, record: bool = False, **env_flags):
    """One deterministic episode per seed, all at once -> (rewards list[float], steps list[int])
    [+ actions int64[T, n] when record: the actions taken, for replay checks]."""
    from .actor_critic import MLPActorCritic

    seeds = [int(s) for s in seeds]
    n = len(seeds)
    env = MerlinVecEnv(n, difficulty=difficulty, size=size, device=device, max_steps=max_steps, seeds=seeds,
                       **env_flags)
    # an MLP policy (observation.flatten) takes the flattened view its input width names: the RGB partial view
    # (9,408) or the encoded full grid (size * size * 3, observation.fully_observable)
    mlp = isinstance(ac, MLPActorCritic)
    full = mlp and ac.actor[0].in_features == size * size * 3

    def act(obs):
        if not mlp:
            return ac.act_codes(obs, deterministic=True)
        x = env.render_full().reshape(n, -1).float() if full else env.flat_obs(obs)
        return ac.act(x, deterministic=True)

    try:
        obs = env.reset().clone()
        total = torch.zeros(n, dtype=torch.float64, device=env.device)
        steps = torch.zeros(n, dtype=torch.int64, device=env.device)
        done = torch.zeros(n, dtype=torch.bool, device=env.device)
        acts = []
        for _ in range(env.max_steps):
            action, _, _ = act(obs)
            obs, _, term, trunc, info = env.step(action, autoreset=False)
            if record:
                acts.append(action.clone())
            live = ~done
            fin = live & (term | trunc)
            total = torch.where(fin, info["episode_return"], total)
            steps += live.long()
            done |= term | trunc
            if bool(done.all()):
                break
        env.errors()
        out = (total.cpu().tolist(), steps.cpu().tolist())
        if record:
            out = out + (torch.stack(acts).cpu(),)
        return out
    finally:
        env.close()


@torch.no_grad()
def evaluate_zero_shot(ac, seeds, difficulty: str = "mediumhard", size: int = 16, device="cuda",
                       max_steps: int | None = None, gamma: float = 0.995, lam: float = 0.95, **env_flags):
    """(rewards list[float], steps list[int], losses list[float]), one deterministic episode per
    seed, all at once (see the module docstring)."""
    from . import _native as nat

    seeds = [int(s) for s in seeds]
    n = len(seeds)
    env = MerlinVecEnv(n, difficulty=difficulty, size=size, device=device, max_steps=max_steps, seeds=seeds,
                       **env_flags)
    try:
        obs = env.reset().clone()
        total = torch.zeros(n, dtype=torch.float64, device=env.device)
        steps = torch.zeros(n, dtype=torch.int64, device=env.device)
        done = torch.zeros(n, dtype=torch.bool, device=env.device)
        codes, acts, vals, rews = [], [], [], []
        for _ in range(env.max_steps):
            action, _, value = ac.act_codes(obs, deterministic=True)
            codes.append(obs.clone())
            acts.append(action)
            vals.append(value)
            obs, rew, term, trunc, info = env.step(action, autoreset=False)
            rews.append(rew.clone())
            live = ~done
            fin = live & (term | trunc)
            total = torch.where(fin, info["episode_return"], total)
            steps += live.long()
            done |= term | trunc
            if bool(done.all()):
                break
        env.errors()
    finally:
        env.close()
    T = len(acts)
    t_idx = torch.arange(T, device=steps.device).unsqueeze(1)
    valid = t_idx < steps.unsqueeze(0)  # [T, n]: the episode's own steps
    last = (t_idx == (steps - 1).unsqueeze(0)).float()  # done at the episode's last step: its bootstrap is masked
    V = torch.stack(vals).contiguous()
    adv, _ = nat.gae(torch.stack(rews).contiguous(), V, last.contiguous(), torch.zeros(n, device=V.device), gamma, lam)
    # per-episode normalisation (torch.std: unbiased), zeros for a one-step episode
    cnt = steps.clamp_min(1).to(torch.float32)
    a = torch.where(valid, adv, torch.zeros((), device=adv.device))
    mean = a.sum(0) / cnt
    var = torch.where(valid, (adv - mean) ** 2, torch.zeros((), device=adv.device)).sum(0) / (cnt - 1).clamp_min(1)
    adv_n = torch.where((steps > 1).unsqueeze(0), (adv - mean) / (var.sqrt() + 1e-8), torch.zeros((), device=adv.device))
    ret = V + adv_n
    # the episode's observations re-evaluated (policy.evaluate), every valid (t, env) at once
    sel = valid.reshape(-1)
    C = torch.stack(codes).reshape(T * n, -1)[sel]
    A = torch.stack(acts).reshape(-1)[sel]
    new_logp, _, new_v = ac.evaluate_codes(C, A)
    env_of = torch.arange(n, device=sel.device).repeat(T)[sel]
    lp_mean = torch.zeros(n, dtype=torch.float64, device=sel.device).index_add_(0, env_of, new_logp.double()) / cnt
    v_err = torch.zeros(n, dtype=torch.float64, device=sel.device).index_add_(
        0, env_of, ((new_v - ret.reshape(-1)[sel]) ** 2).double()) / cnt
    loss = (-lp_mean + 0.5 * v_err).float()
    return total.cpu().tolist(), steps.cpu().tolist(), loss.cpu().tolist()


def evaluate_policy(ac, difficulty: str = "mediumhard", episodes: int = 3, seed: int | None = None,
                    size: int = 16, device="cuda", max_steps: int | None = None, **env_flags):
    """Returns (rewards list[float], steps list[int]) like the reference's evaluate_policy."""
    base = 0 if seed is None else int(seed)
    return evaluate_seeds(ac, range(base, base + episodes), difficulty=difficulty, size=size, device=device,
                          max_steps=max_steps, **env_flags)


def sweep_checkpoints(model_dir: str, difficulty: str = "mediumhard", tasks: int = 50, size: int = 16,
                      device="cuda", **env_flags):
    """[(path, mean reward, mean steps)] of every *.pth in model_dir, best first
    (src/sweep_checkpoints.py:72-100)."""
    from .checkpoints import load_policy

    seeds = range(SWEEP_SEED_BASE, SWEEP_SEED_BASE + tasks)
    results = []
    for path in sorted(glob.glob(os.path.join(model_dir, "*.pth"))):
        policy = load_policy(path, device)
        rew, st = evaluate_seeds(policy, seeds, difficulty=difficulty, size=size, device=device, **env_flags)
        results.append((path, sum(rew) / len(rew), sum(st) / len(st)))
    results.sort(key=lambda r: r[1], reverse=True)
    return results
