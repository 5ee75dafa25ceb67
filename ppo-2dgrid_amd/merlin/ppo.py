"""PPO with the reference's API (src/ppo.py) and a GPU-resident vectorised hot path.

``PPO(env, lr, gamma, lam, clip_eps, update_epochs, batch_size, minibatch_size,
vf_coef, ent_coef, device)`` with ``collect_rollouts() -> last value``,
``compute_gae(rewards, values, dones, last_value) -> (adv, returns)``,
``update(last_value) -> dict(pi_loss, v_loss, entropy, kl, clipfrac, gradnorm)`` and
``train(total_steps)`` as in src/ppo.py:10-175; ``.ac``, ``.batch_size``,
``.episode_returns``, ``.episode_lengths`` and ``._obs_to_tensor`` as used by
ppo/ppo_train.py.

Env kinds:
  * ``MerlinVecEnv`` (N envs) or ``MerlinEnv`` (N = 1): the vectorised path.  Each
    iteration steps T = batch_size / N times; per step one HIP observation expansion,
    one policy forward (PyTorch) and one HIP env-step kernel that writes reward / done /
    next observation straight into the [T][N] rollout storage.  GAE, the advantage
    moments and the normalisation are HIP kernels; minibatch observations are
    re-expanded from the 32-B codes by index (no 37.6 KB/step f32 frame storage).
    The update evaluates conv2 / conv3 once per distinct receptive-field window of the
    rollout and fc1 + heads once per distinct frame of a minibatch (merlin/windows.py).
  * any other gym-style env: the reference's batch-1 loop with f32 frame storage
    (src/ppo.py:64-105), GAE / normalisation still on the HIP kernels.

Semantics kept from the reference: the env is reset at the start of every rollout
(ppo.py:65), done = terminated or truncated with no bootstrap through truncation
(ppo.py:77,113), returns from the un-normalised advantages (ppo.py:119), unbiased
std normalisation over the whole batch (ppo.py:125), randperm minibatches over the
flattened batch (ppo.py:132-134), unclipped value loss, clip_grad_norm_(0.5), Adam.
Per-minibatch scalars are accumulated on the device and read back once per update
instead of six .item() syncs per minibatch (ppo.py:158-163).
"""
from __future__ import annotations

import time

import warnings

import numpy as np
import torch
import torch.optim as optim

from . import _native as nat
from .actor_critic import CNNActorCritic, MLPActorCritic
from .distributed import DataParallel
from .envs import MerlinEnv, MerlinVecEnv
from .metrics.ppo_metrics import aggregate_ppo_update_metrics
from .rollout_buffer import CodeRolloutBuffer, RolloutBuffer
from .windows import deferred_fc1_wgrad

INV255 = 1.0 / 255.0


class _PPOLoss(torch.autograd.Function):
    """The minibatch loss of src/ppo.py:136-150 from per-distinct-frame logits / values (the
    heads' outputs without their biases) and the heads' biases: one HIP pass (merlin_ppo_loss)
    computes the loss, its gradient per frame and for the biases, and the update statistics
    (added to `stats`); backward only scales the stored gradients."""

    @staticmethod
    def forward(ctx, logits, value, bias_actor, bias_critic, mb, sample_index, actions, logp_old, adv, ret, clip_eps,
                vf_coef, ent_coef, stats):
        loss, dlogits, dvalue, dba, dbc = nat.ppo_loss(
            logits.detach(), value.detach(), mb.offs, mb.order, mb.inv, sample_index, actions, logp_old, adv, ret,
            clip_eps, vf_coef, ent_coef, stats, bias_actor=bias_actor, bias_critic=bias_critic)
        ctx.save_for_backward(dlogits, dvalue, dba, dbc.view_as(bias_critic))
        return loss

    @staticmethod
    def backward(ctx, g):
        return tuple(d * g for d in ctx.saved_tensors) + (None,) * 10


# the acting path's fc1 operand scales: one row per rollout step, all zeroed by one kernel when the rollout starts
# (False: one row zeroed by a kernel before every step -- 256 more launches per captured rollout)
ROLLOUT_SCALE_ROWS = True
# the rollout's draw from the acting GEMM's head partials fused into the env step (merlin_env_act_step; False:
# k_act_draw + merlin_env_step, one launch more per step)
FUSE_ACT_STEP = True
# the env step's fallback pass in the rollout even when the look-ahead slots are refilled after every step (False:
# left out there, round 6 -- no reset can meet an empty slot; MerlinVecEnv.set_step_fallback)
ROLLOUT_STEP_FALLBACK = False


class PPO:
    def __init__(self, env, lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=10,
                 batch_size=2048, minibatch_size=256, vf_coef=0.5, ent_coef=0.01, device="cuda",
                 *, dp: DataParallel | None = None, perm_fn=None, conv1_from_codes: bool = True,
                 dedup: bool = True, windows: bool = True, rollout_graph: bool = True):
        self.env = env
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise nat.MerlinNativeError("merlin.PPO runs its hot path as HIP kernels; pass a GPU device")
        self.gamma, self.lam, self.clip_eps = gamma, lam, clip_eps
        self.update_epochs = update_epochs
        self.minibatch_size = minibatch_size
        self.vf_coef, self.ent_coef = vf_coef, ent_coef
        self.dp = dp if dp is not None else DataParallel()
        self.perm_fn = perm_fn  # tests replay recorded permutations through this hook
        # vectorised path: evaluate conv1 from the tile codes (merlin_conv1_lut_*) instead of
        # expanding 37.6 KB frames and running the generic convolution
        self.conv1_from_codes = conv1_from_codes
        # evaluate each distinct observation of a minibatch once (merlin/dedup.py)
        self.dedup = dedup
        self.last_distinct_frac = None  # distinct frames / samples over the last update
        # conv2 / conv3 once per distinct receptive-field window of the update (merlin/windows.py)
        self.windows = windows
        self.last_num_windows = None
        # after one eager rollout, replay the vectorised rollout as one captured HIP graph
        self.rollout_graph = rollout_graph
        self._graph = None
        # the acting layout (CNNActorCritic.rollout_pack): the all-windows conv3 table, or per-frame conv2 lookups;
        # decided at the first rollout and kept (None = not decided yet)
        self.rollout_all_windows = None
        # look-ahead map refill on the side stream after every `refill_every`-th env step (_rollout_body).  Every
        # step: at the bench state (iterations 6-25) refilling every 4th step left so many slots empty at a second
        # reset that the in-step fallback grew from 4.6 to 23 us per step (rollout 35.3 vs ~31 ms,
        # profiles/r03i_busy_union.txt), though at random init it measured 32.0 vs 33.5 ms (scripts/probe_rollout.py)
        self.refill_every = 1
        # PPO._sgd on the window + x6 path: the minibatch step with its launches written out (merlin/fast_step.py;
        # False = the same kernels through the autograd engine)
        self.fast_step = True
        self.stage_impl = "hip"  # the fast step's conv tables: csrc/merlin_stage.hip, or "torch" (autograd's arithmetic)
        self._wstep = None
        # acting draws: counter-based (merlin_act_heads), keyed by this seed (torch.manual_seed's,
        # read without consuming the RNG), the rollout counter below (bumped inside the captured
        # graph: every replay draws afresh), the step and the GLOBAL env index (env_offset + i):
        # ranks of a data-parallel run draw independently, exactly as one process over the
        # concatenated envs would
        self._act_seed = int(torch.initial_seed())
        self._act_epoch = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.episode_returns: list[float] = []
        self.episode_lengths: list[int] = []

        self.vec = env.vec if isinstance(env, MerlinEnv) else env if isinstance(env, MerlinVecEnv) else None
        if isinstance(env, MerlinEnv) and (env.fully_observable or env.flatten):
            # the observation options (scenario.yaml observation.*): the reference's generic env loop, an MLP on a
            # flattened observation (src/ppo.py:38-45) or the CNN on the (size, size, 3) grid encoding
            self.vec = None
        act_dim = env.action_space.n
        if self.vec is not None:
            N = self.vec.num_envs
            if batch_size % N:
                raise ValueError(f"batch_size {batch_size} must be a multiple of num_envs {N}")
            self.num_envs, self.k_steps = N, batch_size // N
            self.batch_size = batch_size
            self._full_obs = None
            if getattr(self.vec, "flatten", False):
                # observation.flatten (scenario_creator.py:52-53): the reference's MLP on the flattened observation
                # (src/ppo.py:38-41), N envs at a time -- the RGB view rebuilt from the stored tile codes per
                # minibatch, or the encoded full grid (observation.fully_observable) stored per step
                self.use_cnn = False
                self.obs_shape = tuple(self.vec.observation_space.shape)
                self.ac = MLPActorCritic(self.obs_shape[0], act_dim).to(self.device)
                self.conv1_from_codes = False
                if getattr(self.vec, "fully_observable", False):
                    self._full_obs = torch.empty((self.k_steps + 1, N) + self.obs_shape, dtype=torch.uint8,
                                                 device=self.device)
            elif getattr(self.vec, "fully_observable", False):
                raise ValueError("the full grid without flatten is smaller than CNNActorCritic's receptive field")
            else:
                self.use_cnn = True
                self.obs_shape = (56, 56, 3)
                self.ac = CNNActorCritic(self.obs_shape, act_dim).to(self.device)
            self.buf = CodeRolloutBuffer(self.k_steps, N, self.device)
            self._obs_step = torch.empty((N, 3, 56, 56), dtype=torch.float32, device=self.device)
            self._mb_obs = None
            # look-ahead map refills on a side stream after every step, overlapping the next act
            # (MerlinVecEnv.refill; the env's own every-16-steps refill is switched off)
            self._refill_stream = (torch.cuda.Stream(self.device) if self.device.type == "cuda" and self.use_cnn
                                   else None)
            if self._refill_stream is not None:
                self.vec.set_refill_interval(0)
        else:
            sample_obs, _ = env.reset()
            self.num_envs, self.k_steps, self.batch_size = 1, batch_size, batch_size
            if sample_obs.ndim == 1:
                self.use_cnn = False
                self.obs_shape = (int(np.prod(sample_obs.shape)),)
                self.ac = MLPActorCritic(self.obs_shape[0], act_dim).to(self.device)
            else:
                self.use_cnn = True
                self.obs_shape = sample_obs.shape
                self.ac = CNNActorCritic(self.obs_shape, act_dim).to(self.device)
            self.buffer = RolloutBuffer(batch_size, self.obs_shape, self.device, is_discrete=True)
        # every parameter a view of one flat buffer (merlin/fast_step.py: the weight stage reads it with one
        # indexed gather; done before anything captures parameter addresses)
        from .fast_step import flatten_parameters

        self._flat_params = flatten_parameters(self.ac)
        # torch's fused Adam: one multi-tensor kernel per step instead of the foreach chain (~9)
        self.optimizer = optim.Adam(self.ac.parameters(), lr=lr, fused=True)
        self.dp.attach(self.ac)
        self._params = [p for p in self.ac.parameters() if p.requires_grad]
        # clip_grad_norm_(0.5) + Adam.step() as two HIP launches on the device (merlin/optim.py)
        self._clip_adam = None
        if self.device.type == "cuda":
            from .optim import ClipAdam

            self._clip_adam = ClipAdam(self.optimizer, 0.5)

    # ------------------------------------------------------------------ helpers
    def _obs_to_tensor(self, state):
        """ppo.py:58-62: one frame -> f32 [1, ...] on the device."""
        state_t = torch.as_tensor(np.asarray(state), dtype=torch.float32, device=self.device)
        return state_t.unsqueeze(0) if self.use_cnn else state_t.view(1, -1)

    def _perm(self, n: int, epoch: int) -> torch.Tensor:
        if self.perm_fn is not None:
            return self.perm_fn(n, epoch).to(self.device)
        return torch.randperm(n, device=self.device)

    # ----------------------------------------------------------------- rollouts
    def _params_on_flat(self) -> bool:
        """Every parameter still a view of self._flat_params at its offset (parameter order)."""
        off, base = 0, self._flat_params.data_ptr()
        for p in self.ac.parameters():
            if p.data_ptr() != base + p.element_size() * off:
                return False
            off += p.numel()
        return off == self._flat_params.numel()

    def _rehome_parameters(self) -> None:
        """A parameter was rebound (`p.data = ...`, load_state_dict(assign=True)): put every parameter back on one
        flat buffer (values kept; the Parameter objects, hence the optimizer state, stay the same) and drop what
        captured the old addresses (the rollout graph, the fast step's weight stage)."""
        from .fast_step import flatten_parameters

        torch.cuda.synchronize(self.device)
        self._graph = None
        self._wstep = None
        self._flat_params = flatten_parameters(self.ac)

    def collect_rollouts(self):
        if self.vec is None:
            return self._collect_rollouts_single()
        if not self.use_cnn:
            return self._collect_rollouts_flat()
        if self._graph is not None and not self._params_on_flat():
            self._rehome_parameters()  # the graph would read the old parameter storage: re-capture
        if self._graph is not None:
            self._graph.replay()
        else:
            self._rollout_body()
            if self.rollout_graph and self.conv1_from_codes:
                self._capture_rollout()
        self._record_episodes()
        self.vec.errors()
        if self.rollout_all_windows:
            nat.tower_errors(self.device)  # the compact acting table saw only observations
        lv = self.buf.last_value
        return float(lv[0].item()) if self.num_envs == 1 else lv

    def _rollout_body(self):
        """ppo.py:64-105 for N envs: reset (ppo.py:65: every rollout starts from a fresh
        reset), T x (act -> env step writing into the [T][N] storage), bootstrap value.
        After every `refill_every`-th step the used look-ahead map slots are refilled on a side stream,
        beside the next act (which reads only the obs codes), and joined before the next step.  (A
        refill's ~60 us of map generation is as long as the act beside it, so refilling after every step
        put it on the step's critical path; an env whose slot is still empty when it resets again takes
        the in-step fallback, which changes no result.)"""
        buf, env = self.buf, self.vec
        T = buf.T
        main, side = torch.cuda.current_stream(self.device), self._refill_stream
        every = max(1, int(self.refill_every))
        # refilled after every step and joined before the next: no reset can meet an empty slot, so the step's
        # fallback pass (a graph node per step, ~4 us + its dispatch gap) is left out; errors() would report one
        env.set_step_fallback(ROLLOUT_STEP_FALLBACK or side is None or every != 1)
        env.reset(out=buf.codes[0])
        with torch.no_grad():
            self._act_epoch.add_(1)
            if self.conv1_from_codes and self.rollout_all_windows is None:  # decided once, before any capture
                self.rollout_all_windows = self.ac._use_all_windows((T + 1) * buf.N, self.device)
            pack = (self.ac.rollout_pack(frames=(T + 1) * buf.N, all_windows=self.rollout_all_windows,
                                         steps=T + 1 if ROLLOUT_SCALE_ROWS else None)
                    if self.conv1_from_codes else None)
            pending = False
            # the draw fused into the env step (merlin_env_act_step): one launch fewer per step
            fused = FUSE_ACT_STEP and pack is not None and self.ac.heads_partials_ok(pack)
            for t in range(T):
                if fused:
                    part = self.ac.act_codes_packed(buf.codes[t], pack, step=t, partials=True)
                else:
                    self._act(buf.codes[t], pack, t, out=(buf.actions[t], buf.logprobs[t], buf.values[t]))
                if pending:
                    main.wait_stream(side)
                    pending = False
                if fused:
                    env.act_step_into(part, self.ac.actor[2].bias, self.ac.critic[2].bias,
                                      (buf.actions[t], buf.logprobs[t], buf.values[t]), buf.codes[t + 1],
                                      buf.rewards[t], None, None, buf.dones[t], buf.ep_return[t], buf.ep_length[t],
                                      seed=self._act_seed, epoch=self._act_epoch, step=t)
                else:
                    env.step_into(buf.actions[t], buf.codes[t + 1], buf.rewards[t], None, None, buf.dones[t],
                                  buf.ep_return[t], buf.ep_length[t])
                if side is not None and (t % every == every - 1 or t == T - 1):
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        env.refill()
                    pending = True
            _, _, last_value = self._act(buf.codes[T], pack, T)
            if pending:
                main.wait_stream(side)
            buf.last_value.copy_(last_value)

    def _capture_rollout(self):
        """Record _rollout_body as one HIP graph (torch.cuda.graph; the env and lookup kernels
        launch on the capturing stream through the C ABI).  The action draws are counter-based
        (merlin_act_heads): the graph bumps the rollout counter _act_epoch on the device at the
        start of every replay, so each replay draws afresh.  Storage, env state and weights are
        read in place, so every replay is a fresh rollout with the current weights, launched as
        one graph instead of ~10k kernels."""
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        try:
            with nat.capture_guard(), torch.cuda.graph(g):  # no GC finalisers inside the capture
                self._rollout_body()
        except Exception as e:  # an op this stack cannot capture: keep launching eagerly
            warnings.warn(f"rollout graph capture failed, rollouts stay eager: {e}")
            self.rollout_graph = False
            torch.cuda.synchronize(self.device)
            return
        self._graph = g

    def _act(self, codes, pack, step, out=None):
        if pack is not None:
            return self.ac.act_codes_packed(codes, pack, seed=self._act_seed, epoch=self._act_epoch, step=step,
                                            out=out, env_offset=self.vec.env_offset)
        nat.expand_obs(codes, out=self._obs_step, scale=INV255)
        res = self.ac.act(self._obs_step, prescaled=True)
        if out is not None:
            for dst, src in zip(out, res):
                dst.copy_(src)
        return res

    def _record_episodes(self):
        done = self.buf.dones > 0  # finished episodes in (step, env) order
        rets = self.buf.ep_return[done]
        lens = self.buf.ep_length[done]
        self.episode_returns.extend(rets.cpu().tolist())
        self.episode_lengths.extend(int(x) for x in lens.cpu().tolist())

    def _collect_rollouts_single(self):
        """Reference loop (ppo.py:64-105) for a generic gym env."""
        state, _ = self.env.reset()
        total_steps, ep_return, ep_length = 0, 0.0, 0
        while total_steps < self.batch_size:
            state_t = self._obs_to_tensor(state)
            with torch.no_grad():
                action, logp, value = self.ac.act(state_t, deterministic=False)
            next_state, reward, terminated, truncated, _ = self.env.step(action.item())
            done = terminated or truncated
            self.buffer.add(state_t.squeeze(0), action.squeeze(), logp.squeeze(), value.squeeze(),
                            torch.tensor(reward, dtype=torch.float32, device=self.device),
                            torch.tensor(done, dtype=torch.float32, device=self.device))
            ep_return += reward
            ep_length += 1
            state = next_state
            total_steps += 1
            if done:
                self.episode_returns.append(ep_return)
                self.episode_lengths.append(ep_length)
                state, _ = self.env.reset()
                ep_return, ep_length = 0.0, 0
        with torch.no_grad():
            _, _, v = self.ac.act(self._obs_to_tensor(state))
        return v.item()

    def _flat_obs_at(self, t=None, index=None):
        """The MLP's f32 observations: step t's (all envs) or the flat samples `index` of the rollout."""
        buf = self.buf
        if self._full_obs is not None:
            x = self._full_obs[t] if index is None else self._full_obs[:buf.T].reshape(buf.T * buf.N, -1)[index]
            return x.reshape(x.shape[0], -1).float()
        codes = buf.codes[t] if index is None else buf.flat_codes
        return self.vec.flat_obs(codes, index=index)

    @torch.no_grad()
    def _collect_rollouts_flat(self):
        """ppo.py:64-105 with the MLP on flattened observations (src/ppo.py:38-41), N envs per step: the act is the
        reference's (Categorical sample with torch's RNG), the env step and the auto-reset are the HIP kernels'."""
        buf, env = self.buf, self.vec
        T = buf.T
        env.reset(out=buf.codes[0])
        if self._full_obs is not None:
            env.render_full(out=self._full_obs[0])
        for t in range(T):
            action, logp, value = self.ac.act(self._flat_obs_at(t))
            buf.actions[t].copy_(action)
            buf.logprobs[t].copy_(logp)
            buf.values[t].copy_(value)
            env.step_into(buf.actions[t], buf.codes[t + 1], buf.rewards[t], None, None, buf.dones[t],
                          buf.ep_return[t], buf.ep_length[t])
            if self._full_obs is not None:
                env.render_full(out=self._full_obs[t + 1])
        _, _, last_value = self.ac.act(self._flat_obs_at(T))
        buf.last_value.copy_(last_value)
        self._record_episodes()
        env.errors()
        return buf.last_value

    # ---------------------------------------------------------------------- GAE
    def compute_gae(self, rewards, values, dones, last_value, stats=None):
        """ppo.py:107-120 on the HIP kernel; [T] or [T, N] device tensors."""
        lv = torch.as_tensor(last_value, dtype=torch.float32, device=rewards.device).reshape(-1)
        return nat.gae(rewards.contiguous(), values.contiguous(), dones.contiguous(), lv, self.gamma,
                       self.lam, stats=stats)

    def _advantages(self, rewards, values, dones, last_value, adv_out=None, ret_out=None):
        """GAE + whole-batch normalisation (ppo.py:124-125); across ranks the moments are
        all-reduced first so every rank normalises with the global batch statistics."""
        stats = torch.zeros(3, dtype=torch.float64, device=rewards.device)
        lv = torch.as_tensor(last_value, dtype=torch.float32, device=rewards.device).reshape(-1)
        adv, ret = nat.gae(rewards, values, dones, lv, self.gamma, self.lam, adv=adv_out, ret=ret_out,
                           stats=stats)
        self.dp.allreduce_sum_(stats)
        return nat.adv_normalize(adv, stats), ret

    # ------------------------------------------------------------------- update
    def update(self, last_value=None):
        if self.vec is not None:
            buf = self.buf
            lv = buf.last_value if last_value is None else last_value
            adv_n, ret = self._advantages(buf.rewards, buf.values, buf.dones, lv, buf.adv, buf.returns)
            self.last_adv_normalized = adv_n  # [T][N], for inspection (the update reads it flat)
            B = buf.T * buf.N
            return self._sgd(B, buf.flat_codes, None, buf.actions.reshape(B), buf.logprobs.reshape(B),
                             adv_n.reshape(B), ret.reshape(B))
        states, actions, logp_old, rewards, values_old, dones = self.buffer.get()
        adv_n, ret = self._advantages(rewards, values_old, dones, last_value)
        return self._sgd(states.shape[0], None, states, actions, logp_old, adv_n, ret)

    def _minibatch_obs(self, codes, states, mb_idx):
        if codes is None:
            return states[mb_idx], False
        if not self.use_cnn:  # the flattened observations of the batched MLP path
            return self._flat_obs_at(index=mb_idx), False
        n = mb_idx.numel()
        if self._mb_obs is None or self._mb_obs.shape[0] < n:
            self._mb_obs = torch.empty((n, 3, 56, 56), dtype=torch.float32, device=self.device)
        out = self._mb_obs[:n]
        nat.expand_obs(codes, index=mb_idx, out=out, scale=INV255)
        return out, True

    def _sgd(self, B, codes, states, actions, logp_old, adv, returns):
        totals = torch.zeros(6, dtype=torch.float64, device=self.device)
        nb = 0
        use_codes = codes is not None and self.conv1_from_codes
        groups = plan = None
        if use_codes and self.dedup:
            from .dedup import FrameGroups

            groups = FrameGroups(codes)
            if not groups.ok:  # a 64-bit hash collision: evaluate every sample this update
                groups = None
            elif self.windows:
                from .windows import WindowPlan

                plan = WindowPlan(codes, groups)
                self.last_num_windows = plan.num_windows
        distinct = 0
        host_mb = []
        t_host = time.perf_counter()
        perms = [self._perm(B, epoch) for epoch in range(self.update_epochs)]  # drawn in epoch order
        # the window + x6 path's step with its launches written out (merlin/fast_step.py)
        fast = plan is not None and self.fast_step and getattr(self.ac, "fc1_impl", None) in ("x6", "h3")
        if fast and not all(p.requires_grad for p in self.ac.parameters()):
            # the fast step writes a gradient for every parameter (and the optimizer steps every parameter that
            # has one): with a frozen parameter the update takes the autograd path, which leaves it untouched
            fast = False
            for p in self.ac.parameters():
                if not p.requires_grad:
                    p.grad = None
        if fast:
            if self._wstep is None or not self._wstep.valid():
                from .fast_step import WindowStep

                if not self._params_on_flat():
                    self._rehome_parameters()
                self._wstep = WindowStep(self)
            self._wstep.bind_grads()
        # one host read per update for every minibatch's distinct-frame groups (merlin/windows.py)
        all_mbws = plan.update_minibatches(perms, self.minibatch_size, bulk=fast) if plan is not None else None
        for epoch in range(self.update_epochs):
            idxs = perms[epoch]
            mbws = all_mbws[epoch] if all_mbws is not None else None
            for k, start in enumerate(range(0, B, self.minibatch_size)):
                mb_idx = idxs[start:start + self.minibatch_size]
                if plan is not None:
                    # distinct frames only: merlin_ppo_loss sums each frame's samples (mb.offs/order)
                    # and adds the statistics to totals[:5] on the device
                    mbw = mbws[k]
                    distinct += int(mbw.groups.numel())
                    if fast:  # forward + backward; every gradient left in its .grad view
                        self._wstep.step(plan, mbw, mb_idx, actions, logp_old, adv, returns, totals)
                    else:
                        with deferred_fc1_wgrad():  # this loop reads p.grad after loss.backward() only
                            logits, values = self.ac.heads_windows(plan, mbw, head_bias=False)
                        loss = _PPOLoss.apply(logits, values, self.ac.actor[2].bias, self.ac.critic[2].bias, mbw,
                                              mb_idx, actions, logp_old, adv, returns, self.clip_eps, self.vf_coef,
                                              self.ent_coef, totals)
                else:
                    lp_old, a_mb, ret_mb = logp_old[mb_idx], adv[mb_idx], returns[mb_idx]
                    if use_codes:
                        g = groups.minibatch(mb_idx) if groups is not None else None
                        if g is not None:
                            distinct += int(g[0].numel())
                        logp_new, entropy, values = self.ac.evaluate_codes(codes, actions[mb_idx], index=mb_idx,
                                                                           groups=g)
                    else:
                        obs, pre = self._minibatch_obs(codes, states, mb_idx)
                        logp_new, entropy, values = self.ac.evaluate(obs, actions[mb_idx], prescaled=pre)
                    values = values.squeeze(-1)
                    ratio = torch.exp(logp_new - lp_old)
                    surr1 = ratio * a_mb
                    surr2 = torch.clamp(ratio, 1 - self.clip_eps, 1 + self.clip_eps) * a_mb
                    pi_loss = -torch.min(surr1, surr2).mean()
                    v_loss = ((values - ret_mb) ** 2).mean()
                    ent = entropy.mean()
                    loss = pi_loss + self.vf_coef * v_loss - self.ent_coef * ent
                    with torch.no_grad():
                        approx_kl = (lp_old - logp_new).mean()
                        clipfrac = (torch.abs(ratio - 1.0) > self.clip_eps).float().mean()
                        totals[:5] += torch.stack([pi_loss.detach(), v_loss.detach(), ent.detach(), approx_kl,
                                                   clipfrac]).double()
                if not fast:
                    self.dp.zero_grad(self.optimizer)
                    loss.backward()
                self.dp.allreduce_grads()
                if self._clip_adam is not None:
                    grad_norm = self._clip_adam.step()
                else:
                    grad_norm = torch.nn.utils.clip_grad_norm_(self._params, 0.5)
                    self.optimizer.step()
                totals[5:].add_(grad_norm.detach())
                nb += 1
                host_mb.append(time.perf_counter())
        self.last_host_loop_ms = (time.perf_counter() - t_host) * 1e3  # host time to queue the update
        # host time to queue each minibatch's optimizer step (the first one includes the update's planning)
        self.last_host_mb_ms = [(b - a) * 1e3 for a, b in zip([t_host] + host_mb[:-1], host_mb)]
        t = totals.cpu().tolist()
        if groups is not None:
            self.last_distinct_frac = float(distinct) / float(self.update_epochs * B)
        return aggregate_ppo_update_metrics(*t, nb)

    def train(self, total_steps=100_000):
        steps_done = 0
        while steps_done < total_steps:
            last_value = self.collect_rollouts()
            self.update(last_value)
            steps_done += self.batch_size
