"""Batched deterministic evaluation (ppo/ppo_train.py:43-69 evaluate_policy of the reference).

The reference resets its eval env with ``seed = base_seed + ep`` for ep < episodes and runs
each episode to termination/truncation with the argmax policy, one env step per forward.
Here all episodes run at once as one ``MerlinVecEnv`` (env ep seeded base_seed + ep, the
same maps), one batched deterministic forward per step, no auto-reset; finished envs keep
stepping but their results are frozen at their first done.
"""
from __future__ import annotations

import torch

from .envs import MerlinVecEnv


@torch.no_grad()
def evaluate_policy(ac, difficulty: str = "mediumhard", episodes: int = 3, seed: int | None = None,
                    size: int = 16, device="cuda", max_steps: int | None = None, **env_flags):
    """Returns (rewards list[float], steps list[int]) like the reference's evaluate_policy."""
    base = 0 if seed is None else int(seed)
    env = MerlinVecEnv(episodes, difficulty=difficulty, size=size, seed=base, device=device,
                       max_steps=max_steps, **env_flags)
    try:
        obs = env.reset().clone()
        n = episodes
        total = torch.zeros(n, dtype=torch.float64, device=env.device)
        steps = torch.zeros(n, dtype=torch.int64, device=env.device)
        done = torch.zeros(n, dtype=torch.bool, device=env.device)
        for _ in range(env.max_steps):
            action, _, _ = ac.act_codes(obs, deterministic=True)
            obs, rew, term, trunc, _ = env.step(action, autoreset=False)
            live = ~done
            total += torch.where(live, rew.double(), torch.zeros_like(total))
            steps += live.long()
            done |= term | trunc
            if bool(done.all()):
                break
        env.errors()
        return total.cpu().tolist(), steps.cpu().tolist()
    finally:
        env.close()
