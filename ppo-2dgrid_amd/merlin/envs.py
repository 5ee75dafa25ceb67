"""GPU-resident MERLIN MiniGrid environments backed by libmerlin_hip.so.

``MerlinVecEnv``  N independent envs in HBM; the fast path used by ``merlin.PPO``.
                  Observations are kept as packed 7x7 tile-class codes (int32[N, 8],
                  32 B/env) and expanded to the RGB frame only when a consumer needs it.
``MerlinEnv``     single-env gym-style wrapper (uint8[56, 56, 3] observations), the
                  drop-in for ``ScenarioCreator.create_env`` of the reference
                  (src/scenario_creator/scenario_creator.py:35-57).

Seeding contract (the reference's training env is unseeded, SURVEY TL;DR 5):
env i of a vector env with base seed s is reset with ``reset(seed=s + env_offset + i)``
once (numpy Generator(PCG64(SeedSequence(.))) as gymnasium does), then every later
reset -- explicit or automatic on done -- continues that env's PCG64 stream unseeded.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _native as nat


class Discrete:
    """Minimal stand-in for gymnasium.spaces.Discrete (gymnasium is optional)."""

    def __init__(self, n: int):
        self.n = n
        self.shape = ()
        self.dtype = np.int64

    def sample(self):
        return int(np.random.randint(self.n))


class Box:
    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype


# algorithmic bytes per env-step of k_env_step in the rollout configuration:
# action 8 + agent state r/w 32 + wall rows 64 + episode accumulators r/w 24 + obs codes 32
# + reward 4 + done 4
ENV_STEP_BYTES = 168


def _entropy_seed() -> int:
    return int.from_bytes(os.urandom(8), "little") >> 1


class MerlinVecEnv:
    """N MERLIN envs stepped by HIP kernels.

    Args mirror the reference's env construction (difficulty / size from
    src/config/scenario.yaml, max_steps = 4*size^2 by default, base_env.py:32-33)
    plus the wrapper flags: ``stuck_penalty`` (StuckPenaltyWrapper semantics,
    stuck_penalty_wrapper.py:3-57; unwired in the reference, so off by default)
    and ``exploration_bonus`` (not defined by the reference; +``bonus`` the first
    time a cell is entered in an episode).
    """

    def __init__(self, num_envs: int, difficulty: str = "mediumhard", size: int = 16,
                 max_steps: int | None = None, seed: int | None = None, device="cuda",
                 stuck_penalty: bool = False, max_stay: int = 3, penalty: float = -0.1,
                 exploration_bonus: bool = False, bonus: float = 0.01, env_offset: int = 0,
                 seeds=None, reseed_each_reset: bool = False, fully_observable: bool = False, flatten: bool = False):
        if difficulty not in nat.DIFFICULTY_IDS:
            raise ValueError(f"Unknown difficulty: {difficulty}")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise nat.MerlinNativeError("MerlinVecEnv runs on a GPU device (HIP); got " + str(device))
        self.num_envs = int(num_envs)
        self.difficulty = difficulty
        self.size = int(size)
        self.max_steps = int(max_steps) if max_steps else 4 * self.size * self.size
        self.env_offset = int(env_offset)
        self.action_space = Discrete(3)
        # the observation wrappers of scenario_creator.py:45-53 (observation.fully_observable / flatten): the step
        # always produces the RGB partial view's tile codes; flat_obs() gives the wrapped observation of a batch --
        # the RGB view (56, 56, 3) or the encoded full grid (size, size, 3), flattened to a vector with flatten
        self.fully_observable, self.flatten = bool(fully_observable), bool(flatten)
        shape = (self.size, self.size, 3) if self.fully_observable else (56, 56, 3)
        if self.flatten:
            shape = (int(np.prod(shape)),)
        self.single_observation_space = Box(0, 255, shape, np.uint8)
        self.observation_space = self.single_observation_space
        cfg = nat.EnvConfig(self.num_envs, self.size, nat.DIFFICULTY_IDS[difficulty], self.max_steps,
                            int(stuck_penalty), int(max_stay), float(penalty), int(exploration_bonus),
                            float(bonus), int(reseed_each_reset))
        self._lib = nat.lib()
        nat.drain_deferred()  # releases queued by a capture outside capture_guard (merlin._native.defer_release)
        with torch.cuda.device(self.device):
            h = C.c_void_p()
            nat.check(self._lib.merlin_env_create(C.byref(cfg), C.byref(h)), "merlin_env_create")
        self._h = h
        self._seed_pending = seed
        self._seeded_once = False
        if seeds is not None:
            self.seed_each(seeds)
        self.obs = torch.zeros((self.num_envs, nat.OBS_WORDS), dtype=torch.int32, device=self.device)
        # per-step scratch outputs for the gym-style step()
        n = self.num_envs
        self._rew = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._term = torch.zeros(n, dtype=torch.uint8, device=self.device)
        self._trunc = torch.zeros(n, dtype=torch.uint8, device=self.device)
        self._epr = torch.zeros(n, dtype=torch.float64, device=self.device)
        self._epl = torch.zeros(n, dtype=torch.int32, device=self.device)

    def close(self):
        """Release the env's device state (merlin_env_destroy: hipFree).  While a HIP-graph capture is open
        (e.g. this env dropped by a GC pass inside another agent's capture) the release waits for it to end:
        a hipFree inside a capture invalidates it (merlin._native.capture_guard)."""
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            lib_ = self._lib
            nat.defer_release(lambda: lib_.merlin_env_destroy(h))

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def seed(self, seed: int) -> None:
        seeds = (np.arange(self.num_envs, dtype=np.uint64) + np.uint64(self.env_offset)
                 + np.uint64(seed))
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_seed(self._h, seeds.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                self.num_envs, self._stream), "merlin_env_seed")
        self._seeded_once = True

    def set_base_seed(self, seed: int) -> None:
        """Seed the next reset() that is given no seed with base `seed` (env i: seed + env_offset + i),
        as the constructor's `seed` does: for callers holding an env from a factory that, like the
        reference's create_env, ignores its seed argument (ppo_train.py's single env)."""
        self._seed_pending = int(seed)
        self._seeded_once = False

    def seed_each(self, seeds) -> None:
        """Seed env i with seeds[i] (e.g. FOMAML task seeds)."""
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64))
        assert seeds.shape == (self.num_envs,)
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_seed(self._h, seeds.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                self.num_envs, self._stream), "merlin_env_seed")
        self._seeded_once = True

    def reset(self, seed: int | None = None, mask: torch.Tensor | None = None, out: torch.Tensor | None = None):
        """Reset all envs (or those with mask != 0).  Returns the obs codes int32[N, 8]."""
        if seed is None and not self._seeded_once:
            seed = self._seed_pending if self._seed_pending is not None else _entropy_seed()
        if seed is not None:
            self.seed(seed)
        out = self.obs if out is None else out
        if mask is not None:
            mask = mask.to(torch.uint8).contiguous()
            # keep untouched rows of `out` equal to the current obs
            if out.data_ptr() != self.obs.data_ptr():
                out.copy_(self.obs)
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_reset(self._h, nat.ptr(mask), nat.ptr(out), self._stream),
                      "merlin_env_reset")
        if out.data_ptr() != self.obs.data_ptr():
            self.obs.copy_(out)
        return out

    def step_into(self, actions: torch.Tensor, obs_out: torch.Tensor | None = None, reward=None, term=None,
                  trunc=None, done=None, ep_return=None, ep_length=None, n_steps: int = 1,
                  action_stride: int | None = None, autoreset: bool = True) -> None:
        """Low-level step writing straight into caller buffers (rollout storage).

        For n_steps > 1, row t of every output is [t*N:(t+1)*N] and actions are read at
        t*action_stride + i (state stays on chip across the steps)."""
        assert actions.dtype == torch.int64 and actions.is_contiguous()
        stride = self.num_envs if action_stride is None else int(action_stride)
        with torch.cuda.device(self.device), nat.KernelTimer.span("k_env_step", self.num_envs * n_steps * ENV_STEP_BYTES):
            nat.check(self._lib.merlin_env_step(
                self._h, nat.ptr(actions), int(n_steps), stride, nat.ptr(obs_out), nat.ptr(reward),
                nat.ptr(term), nat.ptr(trunc), nat.ptr(done), nat.ptr(ep_return), nat.ptr(ep_length),
                int(bool(autoreset)), self._stream), "merlin_env_step")

    def act_step_into(self, part: torch.Tensor, b_actor: torch.Tensor, b_critic: torch.Tensor, out, obs_out=None,
                      reward=None, term=None, trunc=None, done=None, ep_return=None, ep_length=None,
                      deterministic: bool = False, seed: int = 0, epoch=None, step: int = 0) -> None:
        """act -> step in one launch (merlin_env_act_step): the actions drawn from the acting GEMM's head partials
        part f32[2, P, N, 4] (merlin._native.h3_gemm_nt_heads(partials_only=True)) exactly as merlin._native.act_draw
        draws them, written to out = (action, logp, value), then one auto-reset step into the other buffers."""
        action, logp, value = out
        P = int(part.shape[1])
        A = int(b_actor.numel())
        assert part.dtype == torch.float32 and part.is_contiguous() and part.shape == (2, P, self.num_envs, 4)
        assert action.dtype == torch.int64 and action.numel() == logp.numel() == value.numel() == self.num_envs
        assert b_critic.numel() == 1 and 1 <= A <= 4
        if not deterministic and epoch is None:
            raise ValueError("act_step_into: a sampled action needs an epoch counter tensor (int64[1] on the device)")
        with torch.cuda.device(self.device), nat.KernelTimer.span("k_env_step", self.num_envs * ENV_STEP_BYTES):
            nat.check(self._lib.merlin_env_act_step(
                self._h, nat.ptr(part), P, nat.ptr(b_actor), nat.ptr(b_critic), A, int(bool(deterministic)),
                int(seed) & 0xFFFFFFFFFFFFFFFF, nat.ptr(epoch), int(step), int(self.env_offset), nat.ptr(action),
                nat.ptr(logp), nat.ptr(value), nat.ptr(obs_out), nat.ptr(reward), nat.ptr(term), nat.ptr(trunc),
                nat.ptr(done), nat.ptr(ep_return), nat.ptr(ep_length), self._stream), "merlin_env_act_step")

    def set_refill_interval(self, every: int) -> None:
        """Refill the used look-ahead map slots every `every` step calls (default 16); 0 leaves the
        refills to the caller's refill() (merlin_env_set_refill_interval)."""
        nat.check(self._lib.merlin_env_set_refill_interval(self._h, int(every)), "merlin_env_set_refill_interval")

    def set_step_fallback(self, on: bool) -> None:
        """on=False: the caller refills every used look-ahead slot after every step (refill(), refill interval 0),
        so the per-step fallback pass is not launched; a reset that meets an empty slot then raises
        DEVERR_SLOT_EMPTY in errors() (merlin_env_set_step_fallback)."""
        nat.check(self._lib.merlin_env_set_step_fallback(self._h, 1 if on else 0), "merlin_env_set_step_fallback")

    def refill(self) -> None:
        """Generate the next map of every env whose look-ahead slot was used, on the current stream
        (merlin_env_refill).  Touches only the slots and reads the envs' RNG: it may run on a side
        stream beside work that does not step this env, joined before the next step."""
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_refill(self._h, self._stream), "merlin_env_refill")

    def step(self, actions: torch.Tensor, autoreset: bool = True):
        """gym-vector style step: returns (obs codes, reward, terminated, truncated, info).

        With autoreset the obs of a finished env is already the first obs of its next
        episode (src/ppo.py:93-98 resets on done before the next act)."""
        actions = actions.to(device=self.device, dtype=torch.int64).contiguous()
        self.step_into(actions, self.obs, self._rew, self._term, self._trunc, None, self._epr, self._epl,
                       autoreset=autoreset)
        info = {"episode_return": self._epr, "episode_length": self._epl}
        return self.obs, self._rew, self._term.bool(), self._trunc.bool(), info

    # -- observation rendering ------------------------------------------------
    def render_obs(self, codes: torch.Tensor | None = None, index: torch.Tensor | None = None,
                   out: torch.Tensor | None = None, scale: float = 1.0, layout: str = "nchw"):
        codes = self.obs if codes is None else codes
        return nat.expand_obs(codes.reshape(-1, nat.OBS_WORDS), index=index, out=out, scale=scale,
                              layout=layout)

    def render_rgb(self, codes: torch.Tensor | None = None) -> torch.Tensor:
        codes = self.obs if codes is None else codes
        return nat.expand_obs_u8(codes.reshape(-1, nat.OBS_WORDS))

    def flat_obs(self, codes: torch.Tensor | None = None, index: torch.Tensor | None = None) -> torch.Tensor:
        """f32 [n, D]: FlattenObservation of the wrapped observation as the reference's MLP path takes it (src/ppo.py:
        58-62: the uint8 values as floats, no scaling) -- the RGB partial view expanded from tile codes (rows `index`
        of `codes`, default the current ones), D = 9,408."""
        codes = self.obs if codes is None else codes
        return nat.expand_obs_u8(codes.reshape(-1, nat.OBS_WORDS), index=index).view(-1, 56 * 56 * 3).float()

    def render_full(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """uint8[N, size, size, 3]: the fully observable observation of every env's current state
        (observation.fully_observable: FullyObsWrapper + ImgObsWrapper, src/scenario_creator/scenario_creator.py:45-50),
        out[i, x, y] = (object, color, state) of cell (x, y) as minigrid's Grid.encode, the agent's cell (10, 0, dir)
        (merlin_env_full_obs)."""
        S = self.size
        if out is None:
            out = torch.empty((self.num_envs, S, S, 3), dtype=torch.uint8, device=self.device)
        assert out.dtype == torch.uint8 and out.is_contiguous() and out.numel() == self.num_envs * S * S * 3
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_full_obs(self._h, nat.ptr(out), self._stream), "merlin_env_full_obs")
        return out

    # -- introspection (host syncs; tests / tooling) --------------------------
    def get_state(self) -> dict:
        n, S = self.num_envs, self.size
        walls = np.zeros((n, S), dtype=np.uint32)
        agent = np.zeros((n, 8), dtype=np.int32)
        rng = np.zeros((n, 5), dtype=np.uint64)
        vp = C.c_void_p
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_get_state(self._h, walls.ctypes.data_as(vp), agent.ctypes.data_as(vp),
                                                     rng.ctypes.data_as(vp), self._stream), "merlin_env_get_state")
        cells = ((walls[:, :, None] >> np.arange(S, dtype=np.uint32)[None, None, :]) & 1).astype(np.uint8)
        cells[np.arange(n), agent[:, 5], agent[:, 4]] = np.where(
            cells[np.arange(n), agent[:, 5], agent[:, 4]] == 0, 2, cells[np.arange(n), agent[:, 5], agent[:, 4]])
        return {"walls": walls, "cells": cells, "agent_pos": agent[:, 0:2].copy(), "agent_dir": agent[:, 2].copy(),
                "step_count": agent[:, 3].copy(), "goal_pos": agent[:, 4:6].copy(), "stay": agent[:, 6].copy(),
                "rng": rng}

    def errors(self, raise_on_error: bool = True):
        flags, fb = C.c_uint32(), C.c_uint32()
        with torch.cuda.device(self.device):
            nat.check(self._lib.merlin_env_errors(self._h, C.byref(flags), C.byref(fb), self._stream),
                      "merlin_env_errors")
        if raise_on_error and flags.value:
            what = []
            if flags.value & nat.DEVERR_BAD_ACTION:
                what.append("action outside {0,1,2} (ThreeActionWrapper IndexError; -1 = the policy's "
                            "logits were non-finite, merlin_act_heads)")
            if flags.value & nat.DEVERR_PLACE_OBJ:
                what.append("place_obj rejection sampling failed (RecursionError)")
            if flags.value & nat.DEVERR_SLOT_EMPTY:
                what.append("a reset met an empty look-ahead map slot with the step fallback off (refill() was not "
                            "run after every step)")
            raise nat.MerlinNativeError("device env error: " + "; ".join(what))
        return flags.value, fb.value


class MerlinEnv:
    """Single MERLIN env with the gymnasium API the reference's PPO uses:
    ``reset(seed=None) -> (uint8[56,56,3], {})`` and
    ``step(a) -> (obs, float reward, bool terminated, bool truncated, {})``.

    Backed by a 1-env ``MerlinVecEnv`` (no auto-reset: the caller resets on done,
    as src/ppo.py:93-98 does).  Every step crosses the host boundary, like the
    reference on a GPU device (src/ppo.py:59,76); use ``MerlinVecEnv`` for speed.
    """

    def __init__(self, difficulty: str = "mediumhard", size: int = 16, device="cuda", fully_observable: bool = False,
                 flatten: bool = False, **kw):
        self.vec = MerlinVecEnv(1, difficulty=difficulty, size=size, device=device, **kw)
        self.action_space = self.vec.action_space
        # the reference's observation options (src/config/scenario.yaml observation.*,
        # src/scenario_creator/scenario_creator.py:45-53): the RGB partial view (default) or the encoded full grid,
        # either flattened to a vector by FlattenObservation
        self.fully_observable, self.flatten = bool(fully_observable), bool(flatten)
        shape = (self.vec.size, self.vec.size, 3) if self.fully_observable else (56, 56, 3)
        if self.flatten:
            shape = (int(np.prod(shape)),)
        self.observation_space = Box(0, 255, shape, np.uint8)
        self.max_steps = self.vec.max_steps
        self._done = True

    @property
    def unwrapped(self):
        return self

    @property
    def agent_pos(self):
        return tuple(int(v) for v in self.vec.get_state()["agent_pos"][0])

    def _frame(self) -> np.ndarray:
        img = self.vec.render_full() if self.fully_observable else self.vec.render_rgb()
        img = img[0].cpu().numpy()
        return img.reshape(-1) if self.flatten else img

    def reset(self, seed: int | None = None, options=None):
        if seed is not None:
            self.vec.seed(int(seed) - self.vec.env_offset)
        self.vec.reset()
        self._done = False
        return self._frame(), {}

    def step(self, action):
        a = torch.tensor([int(action)], dtype=torch.int64, device=self.vec.device)
        _, rew, term, trunc, _ = self.vec.step(a, autoreset=False)
        flags, _ = self.vec.errors(raise_on_error=False)
        if flags & nat.DEVERR_BAD_ACTION:
            raise IndexError(f"action {action} is not in ThreeActionWrapper's {{0, 1, 2}}")
        r = float(rew[0].item())
        return self._frame(), r, bool(term[0].item()), bool(trunc[0].item()), {}

    def close(self):
        self.vec.close()
