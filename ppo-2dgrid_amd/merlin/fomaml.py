"""First-order MAML over MERLIN tasks (src/fomaml.py of the reference), batched over tasks.

Reference semantics kept (src/fomaml.py:9-223):
  * a task = one map seed; ``collect_trajectory`` resets the env with ``seed=task_seed`` at
    the start and after every done (:63,92), so every episode replays the same map --
    here a MerlinVecEnv with one env per task and ``reseed_each_reset``;
  * inner loop: fast policy = copy of the meta policy, support rollout of k steps, loss =
    PPO clipped surrogate + 0.5 value MSE - 0.05 entropy with GAE(gamma .995, lam .95),
    advantages normalised per task and returns = values + *normalised* advantages
    (:110-156), clip_grad_norm_(0.5), one SGD(lr_inner) step (:176-182);
  * query rollout with the adapted policy, its loss gradient added into the meta
    gradient (:187-202); meta gradient / n_tasks, clip_grad_norm_(0.5), Adam(lr_outer)
    (:207-212); returns (avg query loss, avg query episode reward, avg query episode
    length, the last task's query stats) (:214-223).
MI355X batching: every task's policy is a set of stacked tensors [G, *shape] (merlin.batched_policy
.stack_params) run on the tile-code path with one tower pair per task (merlin.grouped_policy: per-task
conv2 tables, grouped table lookups, batched GEMMs), so both rollouts, the inner step and the query
gradients of all tasks are single batched launches; GAE is the HIP kernel ([k][tasks] layout).  Each
rollout (reset + k x (act -> env step) + bootstrap value) is recorded once as a HIP graph and replayed
with the weights refreshed in place; the draws are the Gumbel-max form of Categorical(logits).sample()
on torch's generator (every replay draws afresh).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.optim as optim

from . import _native as nat
from . import batched_policy as bp
from . import grouped_policy as gp
from .actor_critic import CNNActorCritic
from .envs import MerlinVecEnv

# the rollouts' acting step through merlin_group_act + merlin_env_act_step (False: grouped_policy.act_packed)
FUSED_ACT = True
# after CAPTURE_AFTER eager meta steps of a (tasks, k_support, k_query) shape, its inner step (support loss, every
# task's gradient, per-task clip, SGD) and outer step (query loss, meta gradient, clip, Adam) are recorded as two HIP
# graphs and replayed: ~330 small launches per meta step that the host queued while the GPU idled (round 6)
CAPTURE_STEPS = True
CAPTURE_AFTER = 2


class FOMAML:
    def __init__(self, scenario_creator, lr_inner=0.01, lr_outer=3e-4, device="cuda", difficulty="medium"):
        self.sc = scenario_creator
        self.difficulty = difficulty
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise nat.MerlinNativeError("merlin.FOMAML runs its rollouts/GAE as HIP kernels; pass a GPU device")
        self.lr_inner = lr_inner
        self.env_kwargs = self.sc._env_kwargs(difficulty)
        self.meta_policy = CNNActorCritic((56, 56, 3), 3).to(self.device)
        # capturable: the step count lives on the device, so the Adam step can be part of a captured graph
        self.meta_optimizer = optim.Adam(self.meta_policy.parameters(), lr=lr_outer, capturable=True)
        self.capture_steps = CAPTURE_STEPS
        self._steps = {}  # per (tasks, k_support, k_query): eager step count, then the captured inner / outer graphs
        self.gamma, self.lam = 0.995, 0.95
        self.vf_coef, self.ent_coef, self.clip_eps = 0.5, 0.05, 0.2
        self._env = None
        self._task_seeds = None
        self._rollouts = {}  # per rollout kind: storage, weight pack and its captured HIP graph
        self.rollout_graph = True
        # the acting step as merlin_group_act + merlin_env_act_step (two library launches + the draw fused into the
        # env step) instead of grouped_policy.act_packed (~15 torch / library launches) + merlin_env_step; the draws
        # are counter-based (keyed by this seed, the rollout counter, the step and the task's env), so a captured
        # rollout draws afresh on every replay once the counter is bumped inside it
        self.fused_act = FUSED_ACT
        self._act_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self._act_epoch = torch.zeros(1, dtype=torch.int64, device=self.device)

    # ------------------------------------------------------------------ envs
    def _task_env(self, task_seeds) -> MerlinVecEnv:
        G = len(task_seeds)
        if self._env is None or self._env.num_envs != G:
            if self._env is not None:
                self._env.close()
            self._env = MerlinVecEnv(G, device=self.device, reseed_each_reset=True, **self.env_kwargs)
        self._task_seeds = np.asarray(task_seeds, dtype=np.uint64)
        self._env.seed_each(self._task_seeds)
        return self._env

    # ------------------------------------------------------------ rollouts
    def _rollout_state(self, key, G, steps, params):
        st = self._rollouts.get(key)
        if st is not None and st["G"] == G and st["steps"] == steps:
            return st
        dev = self.device
        st = {"G": G, "steps": steps, "graph": None,
              "codes": torch.zeros((steps + 1, G, 8), dtype=torch.int32, device=dev),
              "act": torch.zeros((steps, G), dtype=torch.int64, device=dev),
              "logp": torch.zeros((steps, G), dtype=torch.float32, device=dev),
              "val": torch.zeros((steps, G), dtype=torch.float32, device=dev),
              "rew": torch.zeros((steps, G), dtype=torch.float32, device=dev),
              "done": torch.zeros((steps, G), dtype=torch.float32, device=dev),
              "epr": torch.zeros((steps, G), dtype=torch.float64, device=dev),
              "epl": torch.zeros((steps, G), dtype=torch.int32, device=dev),
              "last": torch.zeros(G, dtype=torch.float32, device=dev),
              "pack": gp.pack(params),
              "part": torch.zeros((2, 8, G, 4), dtype=torch.float32, device=dev),
              "a3ws": torch.zeros((2 * G, 576), dtype=torch.float32, device=dev),
              "zb": torch.zeros(4, dtype=torch.float32, device=dev)}
        self._rollouts[key] = st
        return st

    def _rollout_body(self, env, st):
        steps = st["steps"]
        pk = st["pack"]
        # the library's own look-ahead refills (every 16 steps) and fallback pass.  (Refilling on a side stream after
        # every step without the fallback, as PPO's rollout does, made these 32-env rollouts slower: 13.5 / 15.4
        # against 9.7 / 11.8 ms for the support / query rollout, profiles/r06f_fomaml_phases.log -- at 32 envs the
        # cross-stream joins cost more than the fallback launch)
        env.reset(out=st["codes"][0])  # = env.reset(seed=task_seed) for every task
        if self.fused_act:
            self._act_epoch.add_(1)  # a fresh draw on every replay
            A = int(pk["ba_r"].shape[1])
            for t in range(steps):
                part = gp.act_parts(pk, st["codes"][t], part=st["part"], a3_ws=st["a3ws"])
                env.act_step_into(part, st["zb"][:A], st["zb"][:1], (st["act"][t], st["logp"][t], st["val"][t]),
                                  st["codes"][t + 1], st["rew"][t], None, None, st["done"][t], st["epr"][t],
                                  st["epl"][t], seed=self._act_seed, epoch=self._act_epoch, step=t)
            part = gp.act_parts(pk, st["codes"][steps], part=st["part"], a3_ws=st["a3ws"])
            st["last"].copy_(part[1, :, :, 0].sum(0))
            return
        for t in range(steps):
            gp.act_packed(pk, st["codes"][t], out=(st["act"][t], st["logp"][t], st["val"][t]))
            env.step_into(st["act"][t], st["codes"][t + 1], st["rew"][t], None, None, st["done"][t], st["epr"][t],
                          st["epl"][t])
        _, _, last = gp.act_packed(pk, st["codes"][steps])
        st["last"].copy_(last)

    @torch.no_grad()
    def collect_trajectory(self, env: MerlinVecEnv, params, steps: int, key: str = "rollout",
                           host_stats: bool = True):
        """k steps of every task in parallel (collect_trajectory, src/fomaml.py:54-108), each task acting
        with its own weights params[name] [G, *shape] (None: the meta policy for every task).  The first
        call per key records the rollout as a HIP graph; later calls refresh the weights in place and
        replay it.  host_stats=False: the episode lists and the env's error flags are not read back (each is a
        host synchronisation; meta_train_step reads the query's once, after everything is queued)."""
        G = env.num_envs
        if params is None:  # the meta policy for every task: one weight set, read by every task's acting step
            W = 1 if self.fused_act else G  # (merlin_group_act shared_weights; the torch path needs G copies)
            params = {n: p.detach().unsqueeze(0).expand(W, *p.shape) for n, p in self.meta_policy.named_parameters()}
        st = self._rollout_state(key, G, steps, params)
        if st["graph"] is None:
            gp.pack_into(st["pack"], params)
            self._rollout_body(env, st)
            if self.rollout_graph:
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                try:
                    with nat.capture_guard(), torch.cuda.graph(g):  # no GC finalisers inside the capture
                        self._rollout_body(env, st)
                    st["graph"] = g
                except Exception:  # keep launching eagerly
                    self.rollout_graph = False
                    torch.cuda.synchronize(self.device)
                # the capture recorded the launches without running them: the rollout returned is a
                # replay (every rollout starts with the reset to the task seeds)
                if st["graph"] is not None:
                    st["graph"].replay()
        else:
            gp.pack_into(st["pack"], params)
            st["graph"].replay()
        out = {"codes": st["codes"], "act": st["act"], "logp": st["logp"], "val": st["val"], "rew": st["rew"],
               "done": st["done"], "last_val": st["last"]}
        if host_stats:
            out.update(self._episode_stats(env, st))
        return out

    @staticmethod
    def _episode_stats(env, st):
        env.errors()
        d = st["done"] > 0
        return {"ep_rews": st["epr"][d].cpu().tolist(), "ep_lens": st["epl"][d].cpu().tolist()}

    # ---------------------------------------------------------------- loss
    def compute_loss(self, batch, params):
        """Per-task losses (compute_loss, src/fomaml.py:110-156) -> (sum over tasks, stats per task)."""
        k, G = batch["rew"].shape
        adv, _ = nat.gae(batch["rew"].contiguous(), batch["val"].contiguous(), batch["done"].contiguous(),
                         batch["last_val"].float().contiguous(), self.gamma, self.lam)
        adv_n = (adv - adv.mean(dim=0, keepdim=True)) / (adv.std(dim=0, keepdim=True) + 1e-8)  # per task
        ret = (batch["val"] + adv_n).detach()
        codes = batch["codes"][:k].transpose(0, 1).reshape(G * k, 8).contiguous()  # task-major
        new_logp, ent, new_val = gp.evaluate(params, codes, k, batch["act"].t())
        old_logp = batch["logp"].t()
        a_t, r_t = adv_n.t(), ret.t()
        ratio = torch.exp(new_logp - old_logp)
        surr1 = ratio * a_t
        surr2 = torch.clamp(ratio, 1.0 - self.clip_eps, 1.0 + self.clip_eps) * a_t
        pi_loss = -torch.min(surr1, surr2).mean(dim=1)
        v_loss = ((new_val - r_t) ** 2).mean(dim=1)
        ent_m = ent.mean(dim=1)
        loss = pi_loss + self.vf_coef * v_loss - self.ent_coef * ent_m  # [G]
        with torch.no_grad():
            kl = (old_logp - new_logp).mean(dim=1)
            clipfrac = (torch.abs(ratio - 1.0) > self.clip_eps).float().mean(dim=1)
        stats = {"loss": loss.detach(), "pi_loss": pi_loss.detach(), "v_loss": v_loss.detach(),
                 "entropy": ent_m.detach(), "kl": kl, "clipfrac": clipfrac}
        return loss.sum(), stats

    @staticmethod
    def _clip_per_task(grads: dict, max_norm: float):
        """clip_grad_norm_ applied to each task's parameter set independently."""
        G = next(iter(grads.values())).shape[0]
        sq = torch.zeros(G, dtype=torch.float32, device=next(iter(grads.values())).device)
        for g in grads.values():
            sq += g.reshape(G, -1).pow(2).sum(dim=1)
        norm = sq.sqrt()
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        return {k: g * coef.view(G, *([1] * (g.dim() - 1))) for k, g in grads.items()}, norm

    # ------------------------------------------------------------ meta step
    def _inner(self, support, G, names):
        """Inner loop (src/fomaml.py:164-185): every fast policy starts as the meta policy; support loss, each task's
        gradient, clip_grad_norm_(0.5) per task, one SGD(lr_inner) step -> the adapted weights [G, *shape]."""
        fast = bp.stack_params(self.meta_policy, G)
        loss_s, _ = self.compute_loss(support, fast)
        grads = dict(zip(names, torch.autograd.grad(loss_s, [fast[n] for n in names])))
        grads, _ = self._clip_per_task(grads, 0.5)
        with torch.no_grad():
            return {n: (fast[n] - self.lr_inner * grads[n]).detach() for n in names}

    def _outer(self, query, adapted, G, names):
        """Outer loop (:187-212): query loss with the adapted weights, the sum of the tasks' gradients / n_tasks as
        the meta gradient, clip_grad_norm_(0.5), Adam.  Returns the query statistics per task."""
        ad = {n: adapted[n].detach().requires_grad_(True) for n in names}
        loss_q, qstats = self.compute_loss(query, ad)
        qgrads = torch.autograd.grad(loss_q, [ad[n] for n in names])
        for (n, p), g in zip(self.meta_policy.named_parameters(), qgrads):
            p.grad = g.sum(dim=0) / G  # sum of the tasks' fast grads / n_tasks (:198-209)
        torch.nn.utils.clip_grad_norm_(self.meta_policy.parameters(), max_norm=0.5)
        self.meta_optimizer.step()
        return qstats

    def _phase(self, st, name, fn, *args):
        """fn(*args) eagerly, or its captured graph (recorded on the call after CAPTURE_AFTER eager meta steps)."""
        g = st.get(name)
        if g is not None:
            g.replay()
            return st[name + "_out"]
        if not (self.capture_steps and st["eager"] >= CAPTURE_AFTER):
            return fn(*args)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        try:
            with nat.capture_guard(), torch.cuda.graph(g):
                out = fn(*args)
        except Exception:  # an op this stack cannot capture: keep launching eagerly
            self.capture_steps = False
            torch.cuda.synchronize(self.device)
            return fn(*args)
        st[name], st[name + "_out"] = g, out
        g.replay()  # the capture recorded the launches without running them
        return out

    def meta_train_step(self, task_seeds, k_support=50, k_query=50):
        G = len(task_seeds)
        env = self._task_env(task_seeds)
        names = [n for n, _ in self.meta_policy.named_parameters()]
        st = self._steps.setdefault((G, k_support, k_query), {"eager": 0})
        if "outer" not in st:
            self.meta_optimizer.zero_grad()
        # inner loop: all fast policies start as the meta policy -> batched support rollout
        # the support rollout's episodes are not reported (:171-176): no host read-back between it and the inner step
        support = self.collect_trajectory(env, None, k_support, key="support", host_stats=False)
        adapted = self._phase(st, "inner", self._inner, support, G, names)
        # outer loop: query rollouts with each task's adapted policy
        query = self.collect_trajectory(env, adapted, k_query, key="query", host_stats=False)
        qstats = self._phase(st, "outer", self._outer, query, adapted, G, names)
        if "outer" in st:  # the captured meta gradient is what .grad shows
            for p, g in zip(self.meta_policy.parameters(), st.setdefault("grads", [p.grad for p in
                                                                                  self.meta_policy.parameters()])):
                p.grad = g
        else:
            st["eager"] += 1
        # the host reads of the meta step, once everything is queued (env error flags: both rollouts')
        query.update(self._episode_stats(env, self._rollouts["query"]))
        avg_loss = float(qstats["loss"].mean().item())
        if query["ep_rews"]:
            avg_rew, avg_steps = float(np.mean(query["ep_rews"])), float(np.mean(query["ep_lens"]))
        else:
            avg_rew, avg_steps = 0.0, float(k_query)
        last = {k: float(v[-1].item()) for k, v in qstats.items() if k != "loss"}
        return avg_loss, avg_rew, avg_steps, last
