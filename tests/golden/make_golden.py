"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (the only place /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Sources, per fixture:
  rng_numpy.npz   numpy's own Generator(PCG64(SeedSequence(s))) (the env RNG of
                  gymnasium seeding.np_random) -- pins the RNG restatements.
  atlas.npz       oracle/tiles.py (numpy restatement of minigrid render_tile).
  env_maps.npz    oracle/minigrid_literal.py with numpy's real Generator: maps
                  after reset(seed) for every generator incl. multi-attempt seeds.
  env_trace.npz   oracle/minigrid_literal.py rollouts (seeded reset, unseeded
                  auto-reset), incl. goal hits and truncation.
  gae_ref.npz     the REFERENCE PPO.compute_gae (src/ppo.py:107-120) and
                  compute_gae_standard (src/utils/utils_rl.py:11-29), imported
                  read-only from /root/reference, plus the adv normalisation of
                  src/ppo.py:125.
  cnn_ref.npz     the REFERENCE CNNActorCritic (src/actor_critic.py) under
                  torch.manual_seed: param checksums + act/evaluate outputs.
  update_ref.npz  one REFERENCE PPO.update (src/ppo.py:122-168) on a small
                  replay batch, with the randperm draws recorded for replay.
  update_rollout_ref.npz  the same on a real single-env rollout of the C oracle's env (repeated
                  observations, episode ends), the fixture the benched update path is pinned to.
  update_grad_ref.npz  the REFERENCE PPO.update at a real minibatch size (8,192-step single-env rollout,
                  minibatches of 2,048) with the first optimizer step's clipped gradient of every tensor
                  and that step's parameter change recorded whole (wrappers around the reference optimizer's
                  step and torch's clip_grad_norm_, defined here).
  fomaml_ref.npz  the REFERENCE FOMAML.compute_loss (src/fomaml.py:110-156) and the
                  per-task inner SGD step + query-gradient accumulation of
                  meta_train_step (:158-212) on recorded support / query batches of
                  3 tasks (the env-free part of a meta step; FOMAML is built with
                  __new__ because its constructor needs minigrid).
The reference code itself is never copied into the repo; only its outputs.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle as O  # noqa: E402
from minigrid_literal import LiteralEnv  # noqa: E402
from tiles import build_atlas  # noqa: E402

REF = "/root/reference"


def gen_rng():
    seeds = [0, 1, 777, 123456, 2**40 + 5]
    out = {"seeds": np.array(seeds, dtype=np.uint64)}
    st = []
    raw = []
    ints_lohi = []
    ints_out = []
    ch_args = []
    ch_out = []
    rs = np.random.RandomState(7)
    for s in seeds:
        g = np.random.PCG64(s)
        S = g.state["state"]
        st.append([S["state"] >> 64, S["state"] & (2**64 - 1), S["inc"] >> 64, S["inc"] & (2**64 - 1)])
        raw.append(g.random_raw(64))
        gen = np.random.default_rng(s)
        lohi = []
        vals = []
        for _ in range(2000):
            lo = int(rs.randint(0, 40))
            hi = lo + int(rs.randint(1, 600))
            lohi.append((lo, hi))
            vals.append(int(gen.integers(lo, hi)))
        ints_lohi.append(lohi)
        ints_out.append(vals)
        gen = np.random.default_rng(s)
        args = []
        outs = np.full((50, 32), -1, dtype=np.int64)
        for i in range(50):
            pop = int(rs.randint(1, 32))
            k = int(rs.randint(1, pop + 1))
            args.append((pop, k))
            outs[i, :k] = gen.choice(pop, size=k, replace=False)
        ch_args.append(args)
        ch_out.append(outs)
    out["state_words"] = np.array(st, dtype=np.uint64)
    out["raw64"] = np.array(raw, dtype=np.uint64)
    out["int_lohi"] = np.array(ints_lohi, dtype=np.int64)
    out["int_out"] = np.array(ints_out, dtype=np.int64)
    out["choice_args"] = np.array(ch_args, dtype=np.int64)
    out["choice_out"] = np.array(ch_out, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "rng_numpy.npz"), **out)


MAP_CASES = [
    ("mediumhard", 16, list(range(0, 40)) + [575, 641, 857, 1600, 777, 123456]),
    ("hard", 16, list(range(0, 12)) + [147, 277]),
    ("hard", 22, list(range(0, 12)) + [429, 1619]),
    ("easy", 16, list(range(0, 8))),
    ("medium", 16, list(range(0, 8))),
    ("hardest", 16, list(range(0, 8)) + [4, 39]),
]


def gen_maps():
    recs = {}
    for diff, size, seeds in MAP_CASES:
        cells = []
        meta = []
        for s in seeds:
            L = LiteralEnv(size, diff)
            codes = L.reset(s)
            cells.append(L.cells())
            meta.append([L.agent_pos[0], L.agent_pos[1], L.agent_dir, L.goal_pos[0], L.goal_pos[1]])
        key = f"{diff}_{size}"
        recs[key + "_seeds"] = np.array(seeds, dtype=np.uint64)
        recs[key + "_cells"] = np.array(cells, dtype=np.uint8)
        recs[key + "_meta"] = np.array(meta, dtype=np.int32)
    np.savez_compressed(os.path.join(HERE, "env_maps.npz"), **recs)


TRACE_CASES = [
    # (difficulty, size, n_envs, T, max_steps, seed_base, p_forward)
    ("mediumhard", 16, 8, 400, 100, 777, 0.6),
    ("hard", 22, 4, 300, 0, 4000, 0.6),
    ("easy", 16, 4, 300, 64, 55, 0.7),
]


def gen_traces():
    recs = {}
    rs = np.random.RandomState(11)
    for diff, size, n, T, max_steps, base, pf in TRACE_CASES:
        seeds = np.arange(base, base + n, dtype=np.uint64)
        p = [(1 - pf) / 2, (1 - pf) / 2, pf]
        acts = rs.choice([0, 1, 2], size=(T, n), p=p).astype(np.int64)
        codes = np.zeros((T + 1, n, 49), np.uint8)
        rew = np.zeros((T, n), np.float32)
        term = np.zeros((T, n), np.uint8)
        trunc = np.zeros((T, n), np.uint8)
        agent = np.zeros((T + 1, n, 4), np.int32)
        for i in range(n):
            L = LiteralEnv(size, diff, max_steps=(max_steps or None))
            c = L.reset(int(seeds[i]))
            codes[0, i] = c.reshape(-1)
            agent[0, i] = (L.agent_pos[0], L.agent_pos[1], L.agent_dir, L.step_count)
            for t in range(T):
                c, r, te, tr = L.step(int(acts[t, i]))
                rew[t, i], term[t, i], trunc[t, i] = np.float32(r), te, tr
                if te or tr:
                    c = L.reset()
                codes[t + 1, i] = c.reshape(-1)
                agent[t + 1, i] = (L.agent_pos[0], L.agent_pos[1], L.agent_dir, L.step_count)
        key = f"{diff}_{size}"
        recs[key + "_cfg"] = np.array([n, T, max_steps, base], dtype=np.int64)
        recs[key + "_actions"] = acts
        recs[key + "_codes"] = codes
        recs[key + "_reward"] = rew
        recs[key + "_term"] = term
        recs[key + "_trunc"] = trunc
        recs[key + "_agent"] = agent
        print(f"trace {key}: terms={int(term.sum())} truncs={int(trunc.sum())}")
    np.savez_compressed(os.path.join(HERE, "env_trace.npz"), **recs)


def _import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from src.actor_critic import CNNActorCritic
    from src.ppo import PPO
    from src.utils.utils_rl import compute_gae_standard

    return PPO, CNNActorCritic, compute_gae_standard


def gen_gae():
    import torch

    PPO, _, gae_std = _import_reference()
    rs = np.random.RandomState(3)
    recs = {}
    for k, (T, p_done) in enumerate([(256, 0.02), (2048, 0.004), (64, 0.3)]):
        r = (rs.rand(T) < 0.05).astype(np.float32) * rs.rand(T).astype(np.float32)
        r -= (rs.rand(T) < 0.1).astype(np.float32) * np.float32(0.1)
        v = rs.randn(T).astype(np.float32)
        d = (rs.rand(T) < p_done).astype(np.float32)
        d[T // 2] = 1.0
        last = float(np.float32(rs.randn()))
        self_ = types.SimpleNamespace(gamma=0.99, lam=0.95)
        adv, ret = PPO.compute_gae(self_, torch.from_numpy(r), torch.from_numpy(v), torch.from_numpy(d), last)
        adv_n = (adv - adv.mean()) / (adv.std() + 1e-8)
        a_std, r_std = gae_std(r, v, d, last, gamma=0.995, lam=0.95)
        recs[f"c{k}_r"], recs[f"c{k}_v"], recs[f"c{k}_d"] = r, v, d
        recs[f"c{k}_last"] = np.float32(last)
        recs[f"c{k}_adv"] = adv.numpy()
        recs[f"c{k}_ret"] = ret.numpy()
        recs[f"c{k}_advnorm"] = adv_n.numpy()
        recs[f"c{k}_adv995"] = a_std.astype(np.float32)
        recs[f"c{k}_ret995"] = np.asarray(r_std, dtype=np.float32)
    recs["ncases"] = np.int64(3)
    np.savez_compressed(os.path.join(HERE, "gae_ref.npz"), **recs)


def _param_checksums(model):
    keys = []
    sums = []
    for name, p in model.state_dict().items():
        keys.append(name)
        t = p.detach().double()
        sums.append([t.sum().item(), t.abs().sum().item(), float(t.reshape(-1)[0].item())])
    return np.array(keys), np.array(sums, dtype=np.float64)


def gen_cnn():
    import torch

    _, CNNActorCritic, _ = _import_reference()
    atlas = build_atlas()
    rs = np.random.RandomState(5)
    codes = rs.randint(0, 4, size=(16, 49)).astype(np.uint8)
    codes[:, 45] = 4  # agent tile at view (3, 6)
    imgs = O.render(codes, atlas)
    torch.manual_seed(0)
    ac = CNNActorCritic((56, 56, 3), 3)
    keys, sums = _param_checksums(ac)
    obs = torch.from_numpy(imgs.astype(np.float32))
    acts = torch.from_numpy(rs.randint(0, 3, size=16).astype(np.int64))
    with torch.no_grad():
        a_det, lp_det, v_det = ac.act(obs, deterministic=True)
        lp_ev, ent_ev, v_ev = ac.evaluate(obs, acts)
        logits = ac.actor(ac.actor_extractor(obs.permute(0, 3, 1, 2)))
    np.savez_compressed(
        os.path.join(HERE, "cnn_ref.npz"),
        seed=np.int64(0), codes=codes, keys=keys, sums=sums, actions=acts.numpy(),
        act_action=a_det.numpy(), act_logp=lp_det.numpy(), act_value=v_det.numpy(),
        ev_logp=lp_ev.numpy(), ev_entropy=ent_ev.numpy(), ev_value=v_ev.numpy(),
        logits=logits.numpy(),
    )


def gen_update():
    import torch

    PPO, _, _ = _import_reference()
    atlas = build_atlas()
    B, MB, EPOCHS = 64, 16, 2
    rs = np.random.RandomState(9)
    codes = rs.randint(0, 4, size=(B, 49)).astype(np.uint8)
    codes[:, 45] = 4
    imgs = O.render(codes, atlas)

    class _StubEnv:  # the reference PPO accepts any gym-like env; only reset/action_space are used
        action_space = types.SimpleNamespace(n=3)

        def reset(self, seed=None):
            return imgs[0].copy(), {}

    torch.manual_seed(0)
    agent = PPO(_StubEnv(), lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=EPOCHS,
                batch_size=B, minibatch_size=MB, vf_coef=0.5, ent_coef=0.05, device="cpu")
    keys, sums0 = _param_checksums(agent.ac)
    actions = rs.randint(0, 3, size=B).astype(np.int64)
    with torch.no_grad():
        lp, _, v = agent.ac.evaluate(torch.from_numpy(imgs.astype(np.float32)), torch.from_numpy(actions))
    rewards = ((rs.rand(B) < 0.1) * rs.rand(B)).astype(np.float32)
    dones = (rs.rand(B) < 0.05).astype(np.float32)
    for t in range(B):
        agent.buffer.add(torch.from_numpy(imgs[t].astype(np.float32)), torch.tensor(actions[t]), lp[t], v[t],
                         torch.tensor(rewards[t]), torch.tensor(dones[t]))
    last_value = float(v[0].item())
    torch.manual_seed(1234)
    perms = np.stack([torch.randperm(B).numpy() for _ in range(EPOCHS)])
    torch.manual_seed(1234)
    stats = agent.update(last_value)
    keys1, sums1 = _param_checksums(agent.ac)
    assert (keys1 == keys).all()
    np.savez_compressed(
        os.path.join(HERE, "update_ref.npz"),
        cfg=np.array([B, MB, EPOCHS], dtype=np.int64), codes=codes, actions=actions,
        logp=lp.numpy(), values=v.numpy(), rewards=rewards, dones=dones,
        last_value=np.float32(last_value), perms=perms, keys=keys, sums0=sums0, sums1=sums1,
        stat_names=np.array(sorted(stats)), stat_vals=np.array([stats[k] for k in sorted(stats)]),
        hparams=np.array([3e-4, 0.99, 0.95, 0.2, 0.5, 0.05]),
    )


def gen_update_rollout():
    """update_rollout_ref.npz: one REFERENCE PPO.update (src/ppo.py:122-168) on a real single-env
    rollout (the C oracle's mediumhard env, seed 777, uniformly random actions, max_steps 48 so that
    episodes end and auto-reset): its observations repeat (turns in place, revisited cells), so the
    distinct-frame grouping and the receptive-field windows of the benched update path are exercised
    on the reference's own numbers.  Values / log-probs from the reference's initial weights."""
    import torch

    PPO, _, _ = _import_reference()
    atlas = build_atlas()
    B, MB, EPOCHS = 1024, 256, 3
    rs = np.random.RandomState(31)
    actions = rs.randint(0, 3, size=(B, 1)).astype(np.int64)
    codes, rew, term, trunc, _ = O.batch_rollout(np.array([777], dtype=np.uint64), actions, max_steps=48)
    codes = codes[:B, 0]
    imgs = O.render(codes, atlas)
    rewards = rew[:, 0].astype(np.float32)
    dones = np.maximum(term, trunc)[:, 0].astype(np.float32)
    actions = actions[:, 0]

    class _StubEnv:
        action_space = types.SimpleNamespace(n=3)

        def reset(self, seed=None):
            return imgs[0].copy(), {}

    torch.manual_seed(0)
    agent = PPO(_StubEnv(), lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=EPOCHS,
                batch_size=B, minibatch_size=MB, vf_coef=0.5, ent_coef=0.05, device="cpu")
    keys, sums0 = _param_checksums(agent.ac)
    with torch.no_grad():
        lp, _, v = agent.ac.evaluate(torch.from_numpy(imgs.astype(np.float32)), torch.from_numpy(actions))
    for t in range(B):
        agent.buffer.add(torch.from_numpy(imgs[t].astype(np.float32)), torch.tensor(actions[t]), lp[t], v[t],
                         torch.tensor(rewards[t]), torch.tensor(dones[t]))
    last_value = float(v[-1].item())
    torch.manual_seed(4321)
    perms = np.stack([torch.randperm(B).numpy() for _ in range(EPOCHS)])
    torch.manual_seed(4321)
    stats = agent.update(last_value)
    keys1, sums1 = _param_checksums(agent.ac)
    assert (keys1 == keys).all()
    np.savez_compressed(
        os.path.join(HERE, "update_rollout_ref.npz"),
        cfg=np.array([B, MB, EPOCHS], dtype=np.int64), codes=codes, actions=actions,
        logp=lp.numpy(), values=v.numpy(), rewards=rewards, dones=dones,
        last_value=np.float32(last_value), perms=perms, keys=keys, sums0=sums0, sums1=sums1,
        stat_names=np.array(sorted(stats)), stat_vals=np.array([stats[k] for k in sorted(stats)]),
        hparams=np.array([3e-4, 0.99, 0.95, 0.2, 0.5, 0.05]),
    )


def gen_update_grad():
    """update_grad_ref.npz: the REFERENCE PPO.update (src/ppo.py:122-168) at a real minibatch size -- an 8,192-step
    single-env rollout of the C oracle's mediumhard env (seed 777, uniformly random actions, the env's own max_steps
    1,024), one epoch of 4 minibatches of 2,048 -- with the FIRST optimizer step's gradient recorded whole: a wrapper
    around the reference optimizer's `step` (after clip_grad_norm_, :153-155) saves every parameter's clipped
    .grad and the parameters' change by that step; a wrapper around torch's clip_grad_norm_ keeps its returned
    (pre-clip) norm.  Nothing in the reference is edited: both wrappers live here, around objects it creates."""
    import torch

    PPO, _, _ = _import_reference()
    atlas = build_atlas()
    B, MB, EPOCHS = 8192, 2048, 1
    rs = np.random.RandomState(47)
    actions = rs.randint(0, 3, size=(B, 1)).astype(np.int64)
    codes, rew, term, trunc, _ = O.batch_rollout(np.array([777], dtype=np.uint64), actions)
    codes = codes[:B, 0]
    imgs = O.render(codes, atlas)
    rewards = rew[:, 0].astype(np.float32)
    dones = np.maximum(term, trunc)[:, 0].astype(np.float32)
    actions = actions[:, 0]

    class _StubEnv:
        action_space = types.SimpleNamespace(n=3)

        def reset(self, seed=None):
            return imgs[0].copy(), {}

    torch.manual_seed(0)
    agent = PPO(_StubEnv(), lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=EPOCHS,
                batch_size=B, minibatch_size=MB, vf_coef=0.5, ent_coef=0.05, device="cpu")
    keys, sums0 = _param_checksums(agent.ac)
    names = [n for n, _ in agent.ac.named_parameters()]
    with torch.no_grad():
        lp, _, v = agent.ac.evaluate(torch.from_numpy(imgs.astype(np.float32)), torch.from_numpy(actions))
    for t in range(B):
        agent.buffer.add(torch.from_numpy(imgs[t].astype(np.float32)), torch.tensor(actions[t]), lp[t], v[t],
                         torch.tensor(rewards[t]), torch.tensor(dones[t]))
    last_value = float(v[-1].item())
    # the advantages the update normalises, as it computes them (src/ppo.py:123-125: the reference's own
    # compute_gae on the buffer, then the fp32 torch moments) -- stored, so a test can feed the benched path the
    # reference's exact normalised advantages (torch's CPU reductions round by the host's vector ISA)
    _, _, _, rw, vo, dn = agent.buffer.get()
    adv_raw, ret_ref = agent.compute_gae(rw, vo, dn, last_value)
    adv_norm = (adv_raw - adv_raw.mean()) / (adv_raw.std() + 1e-8)
    rec = {}
    norms = []
    clip_orig = torch.nn.utils.clip_grad_norm_

    def clip_wrap(*a, **k):
        n = clip_orig(*a, **k)
        norms.append(float(n))
        return n

    step_orig = agent.optimizer.step

    def step_wrap(*a, **k):
        first = not rec
        if first:
            params = [p for _, p in agent.ac.named_parameters()]
            rec["p0"] = [p.detach().clone() for p in params]
            rec["grads"] = [p.grad.detach().clone() for p in params]
        out = step_orig(*a, **k)
        if first:
            rec["delta"] = [p.detach() - p0 for p, p0 in zip(params, rec["p0"])]
        return out

    agent.optimizer.step = step_wrap
    torch.nn.utils.clip_grad_norm_ = clip_wrap
    try:
        torch.manual_seed(4747)
        perms = np.stack([torch.randperm(B).numpy() for _ in range(EPOCHS)])
        torch.manual_seed(4747)
        stats = agent.update(last_value)
    finally:
        torch.nn.utils.clip_grad_norm_ = clip_orig
    keys1, sums1 = _param_checksums(agent.ac)
    assert (keys1 == keys).all() and len(norms) == EPOCHS * (B // MB)
    out = dict(
        cfg=np.array([B, MB, EPOCHS], dtype=np.int64), codes=codes, actions=actions,
        logp=lp.numpy(), values=v.numpy(), rewards=rewards, dones=dones,
        last_value=np.float32(last_value), perms=perms, keys=keys, sums0=sums0, sums1=sums1,
        stat_names=np.array(sorted(stats)), stat_vals=np.array([stats[k] for k in sorted(stats)]),
        hparams=np.array([3e-4, 0.99, 0.95, 0.2, 0.5, 0.05]), param_names=np.array(names),
        first_norm=np.float64(norms[0]), norms=np.array(norms),
        adv_norm=adv_norm.numpy().astype(np.float32), returns=ret_ref.numpy().astype(np.float32),
    )
    for i, (g, d) in enumerate(zip(rec["grads"], rec["delta"])):
        # the starting weights too: torch's orthogonal_ init (QR through the host's LAPACK) rounds differently on
        # another CPU, and at the initial weights the actor tower's gradient is a near-cancelling sum that turns a
        # 1e-7 weight difference into ~6e-4 of gradient -- the test loads these, not a re-run of the init
        out[f"p0_{i}"] = rec["p0"][i].numpy().astype(np.float32)
        out[f"grad{i}"] = g.numpy().astype(np.float32)  # the clipped gradient Adam consumed
        out[f"step{i}"] = (d.double() / 3e-4).numpy().astype(np.float16)  # the first Adam step in units of lr
    np.savez_compressed(os.path.join(HERE, "update_grad_ref.npz"), **out)
    print(f"update_grad_ref: {len(np.unique(codes, axis=0))} distinct frames of {B}, {int(dones.sum())} dones, "
          f"first-step norm {norms[0]:.5f}")


def gen_fomaml():
    import copy

    import torch

    _import_reference()
    from src.actor_critic import CNNActorCritic
    from src.fomaml import FOMAML

    atlas = build_atlas()
    G, K = 3, 24
    rs = np.random.RandomState(21)
    ref = FOMAML.__new__(FOMAML)  # the constructor builds a minigrid env; compute_loss needs none
    ref.device = torch.device("cpu")
    ref.gamma, ref.lam, ref.vf_coef, ref.ent_coef, ref.clip_eps = 0.995, 0.95, 0.5, 0.05, 0.2
    lr_inner = 0.01
    torch.manual_seed(0)
    meta = CNNActorCritic((56, 56, 3), 3)
    keys, sums0 = _param_checksums(meta)

    def batch_of(policy):
        codes = rs.randint(0, 4, size=(K + 1, 49)).astype(np.uint8)
        codes[:, 45] = 4
        imgs = torch.from_numpy(O.render(codes, atlas).astype(np.float32))
        act = torch.from_numpy(rs.randint(0, 3, size=K).astype(np.int64))
        with torch.no_grad():  # what collect_trajectory stores from policy.act (src/fomaml.py:73-86)
            lp, _, v = policy.evaluate(imgs[:K], act)
            _, _, last = policy.act(imgs[K:K + 1])
        rew = ((rs.rand(K) < 0.15) * rs.rand(K)).astype(np.float32)
        done = (rs.rand(K) < 0.1).astype(np.float32)
        done[K // 2] = 1.0
        b = {"obs": imgs[:K], "act": act, "rew": torch.from_numpy(rew), "val": v, "logp": lp,
             "done": torch.from_numpy(done), "last_val": last}
        return codes, b

    rec = {"cfg": np.array([G, K], dtype=np.int64), "lr_inner": np.float64(lr_inner), "keys": keys, "sums0": sums0}
    meta_grad = {n: torch.zeros_like(p) for n, p in meta.named_parameters()}
    meta_sd = copy.deepcopy(meta.state_dict())
    for g in range(G):
        fast = copy.deepcopy(meta)
        fast.load_state_dict(meta_sd)
        sc, sb = batch_of(fast)
        loss_s, st_s = ref.compute_loss(sb, fast)
        inner = torch.optim.SGD(fast.parameters(), lr=lr_inner)
        inner.zero_grad()
        loss_s.backward()
        torch.nn.utils.clip_grad_norm_(fast.parameters(), max_norm=0.5)
        inner.step()
        qc, qb = batch_of(fast)  # the query rollout runs the adapted policy
        loss_q, st_q = ref.compute_loss(qb, fast)
        fast.zero_grad()
        loss_q.backward()
        for n, p in fast.named_parameters():
            meta_grad[n] += p.grad
        for tag, c, b, loss, st in (("s", sc, sb, loss_s, st_s), ("q", qc, qb, loss_q, st_q)):
            rec[f"t{g}_{tag}_codes"] = c
            for k in ("act", "rew", "val", "logp", "done"):
                rec[f"t{g}_{tag}_{k}"] = b[k].numpy()
            rec[f"t{g}_{tag}_last_val"] = np.float32(b["last_val"].item())
            rec[f"t{g}_{tag}_loss"] = np.float64(loss.item())
            rec[f"t{g}_{tag}_stats"] = np.array([st[k] for k in ("pi_loss", "v_loss", "entropy", "kl", "clipfrac")])
    # the meta gradient of meta_train_step before its clip / Adam (:205-209): sum / n_tasks; stored
    # as per-parameter (norm, sum) and 256 fixed sampled elements per parameter
    names, stats, idx, vals = [], [], [], []
    for n, gsum in meta_grad.items():
        gm = (gsum / G).reshape(-1).double()
        names.append(n)
        stats.append([gm.norm().item(), gm.sum().item()])
        sel = np.sort(np.random.RandomState(len(names)).choice(gm.numel(), min(256, gm.numel()), replace=False))
        idx.append(np.pad(sel, (0, 256 - sel.size), constant_values=-1))
        vals.append(np.pad(gm.numpy()[sel], (0, 256 - sel.size)))
    rec.update(grad_names=np.array(names), grad_stats=np.array(stats), grad_idx=np.array(idx, dtype=np.int64),
               grad_vals=np.array(vals))
    np.savez_compressed(os.path.join(HERE, "fomaml_ref.npz"), **rec)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # e.g. `make_golden.py gen_fomaml`: only the named fixtures
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    np.savez_compressed(os.path.join(HERE, "atlas.npz"), atlas=build_atlas())
    gen_rng()
    gen_maps()
    gen_traces()
    gen_gae()
    gen_cnn()
    gen_update()
    gen_update_rollout()
    gen_update_grad()
    gen_fomaml()
    print("golden fixtures written to", HERE)
