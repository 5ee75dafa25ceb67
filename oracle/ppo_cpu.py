"""TEST/BASELINE INFRASTRUCTURE ONLY -- CPU restatement of the reference's training
loop, used as bench.py's ``cpu_baseline`` ("port") and never by the product.

What it restates (reference paths): the batch-1 rollout of PPO.collect_rollouts
(src/ppo.py:64-105) over one MERLIN env (the C oracle env + the RGB frame render,
standing in for minigrid + RGBImgPartialObsWrapper which are absent here), the
Python-loop GAE (ppo.py:107-120, via the C oracle restatement), the whole-batch
advantage normalisation (ppo.py:125) and the update loop (ppo.py:122-168: randperm
minibatches, clipped surrogate, value MSE, entropy bonus, clip_grad_norm_(0.5),
Adam) with the reference's CNN (actor_critic.py) written out with torch.nn on CPU.
Hyper-parameters default to ppo/ppo_train.py:21-31 (ent_coef 0.05).
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np
import torch
import torch.nn as nn

import oracle as O
from tiles import build_atlas


def _ortho(layer, std=np.sqrt(2)):
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, 0.0)
    return layer


def _tower():
    return nn.Sequential(_ortho(nn.Conv2d(3, 32, 8, 4)), nn.ReLU(), _ortho(nn.Conv2d(32, 64, 4, 2)), nn.ReLU(),
                         _ortho(nn.Conv2d(64, 64, 3, 1)), nn.ReLU(), nn.Flatten())


class CpuActorCritic(nn.Module):
    def __init__(self, hidden=512, act_dim=3):
        super().__init__()
        self.fa, self.fc = _tower(), _tower()
        self.pi = nn.Sequential(_ortho(nn.Linear(576, hidden)), nn.ReLU(), _ortho(nn.Linear(hidden, act_dim), 0.01))
        self.v = nn.Sequential(_ortho(nn.Linear(576, hidden)), nn.ReLU(), _ortho(nn.Linear(hidden, 1), 1.0))

    def heads(self, frames_nhwc):
        x = frames_nhwc.permute(0, 3, 1, 2).float() / 255.0
        logits = self.pi(self.fa(x))
        return torch.distributions.Categorical(logits=logits), self.v(self.fc(x)).squeeze(-1)


class CpuEnv:
    def __init__(self, difficulty="mediumhard", size=16):
        L = O.lib()
        L.o_env_new.restype = C.c_void_p
        L.o_env_new.argtypes = [C.c_int, C.c_int, C.c_int]
        L.o_env_free.argtypes = [C.c_void_p]
        L.o_env_reset_codes.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_void_p]
        L.o_env_step_codes.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.o_env_step_codes.restype = C.c_double
        self.L = L
        self.h = L.o_env_new(size, O.DIFFICULTIES[difficulty], 0)
        self.codes = np.zeros(49, dtype=np.uint8)
        self.atlas = build_atlas()

    def _frame(self):
        return O.render(self.codes, self.atlas)[0]

    def reset(self, seed=None):
        self.L.o_env_reset_codes(self.h, int(seed is not None), 0 if seed is None else seed,
                                 self.codes.ctypes.data_as(C.c_void_p))
        return self._frame()

    def step(self, a):
        te, tr = C.c_int(), C.c_int()
        r = self.L.o_env_step_codes(self.h, int(a), self.codes.ctypes.data_as(C.c_void_p), C.byref(te), C.byref(tr))
        return self._frame(), r, bool(te.value), bool(tr.value)


def evaluate(ac, env, episodes=3, seed=0, max_steps=1024):
    """ppo/ppo_train.py:43-69: `episodes` deterministic (argmax) episodes, reset(seed=seed + ep)."""
    for ep in range(episodes):
        state = env.reset(seed + ep)
        for _ in range(max_steps):
            with torch.no_grad():
                dist, _ = ac.heads(torch.from_numpy(state.astype(np.float32))[None])
            state, _, te, tr = env.step(int(dist.probs.argmax(-1).item()))
            if te or tr:
                break


def run_iterations(n_iter=1, batch=2048, mb=256, epochs=10, lr=3e-4, gamma=0.99, lam=0.95, clip=0.2, vf=0.5,
                   ent_coef=0.05, seed=777, difficulty="mediumhard", eval_episodes=0):
    """Returns (env_steps, seconds) for n_iter rollout+GAE+update iterations on CPU; with
    eval_episodes > 0, (env_steps, seconds without the evals, seconds with them): the per-iteration
    deterministic evaluation of ppo/ppo_train.py:150 on its own env (seed + 999)."""
    torch.manual_seed(seed)
    env = CpuEnv(difficulty)
    ac = CpuActorCritic()
    opt = torch.optim.Adam(ac.parameters(), lr=lr)
    frames = torch.zeros((batch, 56, 56, 3))
    acts = torch.zeros(batch, dtype=torch.long)
    logps, vals, rews, dones = (torch.zeros(batch) for _ in range(4))
    state = env.reset(seed)
    eval_env = CpuEnv(difficulty) if eval_episodes else None
    t_eval = 0.0
    t0 = time.perf_counter()
    for _ in range(n_iter):
        state = env.reset()
        for t in range(batch):
            st = torch.from_numpy(state.astype(np.float32))
            with torch.no_grad():
                dist, v = ac.heads(st[None])
                a = dist.sample()
            nxt, r, te, tr = env.step(a.item())
            frames[t], acts[t], logps[t], vals[t] = st, a[0], dist.log_prob(a)[0], v[0]
            rews[t], dones[t] = r, float(te or tr)
            state = env.reset() if (te or tr) else nxt
        with torch.no_grad():
            _, lv = ac.heads(torch.from_numpy(state.astype(np.float32))[None])
        adv, ret = O.gae_tn(rews.numpy(), vals.numpy(), dones.numpy(), lv.numpy(), gamma, lam)
        adv = torch.from_numpy(adv[:, 0])
        ret = torch.from_numpy(ret[:, 0])
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        for _ in range(epochs):
            perm = torch.randperm(batch)
            for s in range(0, batch, mb):
                i = perm[s:s + mb]
                dist, v = ac.heads(frames[i])
                lp = dist.log_prob(acts[i])
                ratio = torch.exp(lp - logps[i])
                pi = -torch.min(ratio * adv[i], torch.clamp(ratio, 1 - clip, 1 + clip) * adv[i]).mean()
                loss = pi + vf * ((v - ret[i]) ** 2).mean() - ent_coef * dist.entropy().mean()
                opt.zero_grad(set_to_none=True)
                loss.backward()
                torch.nn.utils.clip_grad_norm_(ac.parameters(), 0.5)
                opt.step()
        if eval_env is not None:
            te0 = time.perf_counter()
            evaluate(ac, eval_env, eval_episodes, seed + 999)
            t_eval += time.perf_counter() - te0
    total = time.perf_counter() - t0
    if eval_env is not None:
        return n_iter * batch, total - t_eval, total
    return n_iter * batch, total
