"""Rollout storage (src/rollout_buffer.py of the reference, plus the HBM layout of
the vectorised path).

``RolloutBuffer``      the reference's flat per-step buffer (rollout_buffer.py:3-32):
                       states f32[B, *obs_shape], actions, logprobs, rewards, values,
                       dones; used by PPO with a generic (non-MERLIN) gym env.
``CodeRolloutBuffer``  the MERLIN-AMD layout for N envs x T steps, all [T][N]
                       (row t holds every env's step t, so the GAE scan and the env
                       step kernel touch contiguous rows):
                         codes   int32[T+1][N][8]  packed 7x7 tile classes (32 B per
                                                   observation instead of the 37.6 KB
                                                   f32 frame; expanded on demand)
                         actions int64[T][N]; logprobs/values/rewards/dones f32[T][N]
                         adv/returns f32[T][N]; ep_return f64 / ep_length i32 [T][N]
                       At N=4096, T=256: 33.6 MB codes + 4 MB per f32 field.
"""
from __future__ import annotations

import torch


class RolloutBuffer:
    def __init__(self, buffer_size, obs_shape, device, is_discrete=True):
        f32 = dict(dtype=torch.float32, device=device)
        self.states = torch.zeros((buffer_size, *obs_shape), **f32)
        self.actions = torch.zeros(buffer_size, dtype=torch.long if is_discrete else torch.float32,
                                   device=device)
        self.logprobs = torch.zeros(buffer_size, **f32)
        self.rewards = torch.zeros(buffer_size, **f32)
        self.values = torch.zeros(buffer_size, **f32)
        self.dones = torch.zeros(buffer_size, **f32)
        self.max_size = buffer_size
        self.ptr = 0

    def add(self, state, action, logprob, value, reward, done):
        i = self.ptr
        for dst, src in ((self.states, state), (self.actions, action), (self.logprobs, logprob),
                         (self.values, value), (self.rewards, reward), (self.dones, done)):
            dst[i] = src
        self.ptr = (i + 1) % self.max_size

    def get(self):
        self.ptr = 0
        return self.states, self.actions, self.logprobs, self.rewards, self.values, self.dones


class CodeRolloutBuffer:
    def __init__(self, T: int, N: int, device):
        self.T, self.N = int(T), int(N)
        dev = torch.device(device)
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
        self.codes = z(T + 1, N, 8, dt=torch.int32)
        self.actions = z(T, N, dt=torch.int64)
        self.logprobs = z(T, N)
        self.values = z(T, N)
        self.rewards = z(T, N)
        self.dones = z(T, N)
        self.adv = z(T, N)
        self.returns = z(T, N)
        self.ep_return = z(T, N, dt=torch.float64)
        self.ep_length = z(T, N, dt=torch.int32)
        self.stats = z(3, dt=torch.float64)
        self.last_value = z(N)

    @property
    def flat_codes(self) -> torch.Tensor:
        """codes of the T stored observations as [T*N, 8] (flat index t*N + i)."""
        return self.codes[: self.T].reshape(self.T * self.N, 8)
