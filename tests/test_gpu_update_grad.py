"""GPU: the BENCHED update's gradient pinned to the reference's own gradient at a real minibatch size.

`update_grad_ref.npz` (tests/golden/make_golden.py gen_update_grad) holds the reference PPO.update
(src/ppo.py:122-168) on an 8,192-step single-env rollout of the C oracle's mediumhard env, one epoch of four
minibatches of 2,048, with the FIRST optimizer step recorded whole: the starting weights, every parameter's clipped
gradient as clip_grad_norm_ left it for Adam (:153-156), the pre-clip norm, the parameters' change by that step, and
the normalised advantages / returns the update used.

Here the same inputs run through exactly what bench.py times -- code storage, the HIP GAE, the distinct-frame
grouping, conv2 / conv3 once per receptive-field window, fc1's three GEMMs in h3 form over operand planes (k_h3_pqg /
k_h3_pq / k_h3_tq), the fused loss and the two-launch clip + Adam -- from the reference's starting weights, and the
gradient the benched path hands to its optimizer (p.grad at the first ClipAdam.step) is compared tensor by tensor with
the reference's, and both with the same gradient in float64 (the reference's network and loss restated below on the
CPU in double).

Conditioning.  At the initial weights the actor's head is tiny (orthogonal init, std 0.01), so the actor tower's and
the actor fc1's gradients are near-cancelling sums (|g| ~ 1e-5 per weight), and a few ReLU pre-activations sit within
fp32 rounding of zero (one actor fc1 unit at 1.6e-8 of its layer's max): an fp32 forward that sums in another order
may put such a unit on the other side of its kink, which adds or removes that unit's whole gradient contribution --
~6e-4 of the actor tower's gradient (perturbing the weights by 2^-22 relative moves the float64 gradient by as much,
by 2^-24 only ~1e-7).  So every tensor is held to 1e-5 of its norm PLUS the tie envelope: the sum, over the ReLU units
whose float64 pre-activation is within 2^-21 of its sum's absolute mass (sum |a_k w_k| + |b|), of the norm of each
unit's own gradient contribution (its dL/dh times dz/dtheta for its sample, computed in float64 here).  Away from the actor side the envelope is ~0 and the
bound is the plain 1e-5; the reference's own fp32 gradient is within ~2.5e-6 of float64 at these weights.

The advantages: the reference normalises them with fp32 torch moments (src/ppo.py:125), the benched path with f64
moments (the GAE itself is bit-exact); the first test injects the reference's normalised advantages and returns, the
second runs the benched path's own and compares with float64 on those."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REL = 1e-5  # per-tensor relative norm of the gradient difference, on top of the ReLU-tie envelope


# a ReLU pre-activation z = sum_k a_k w_k + b is a tie at fp32 precision when |z| <= TIE * (sum_k |a_k w_k| + |b|):
# within ~log2(K) units of fp32 rounding of the sum's absolute mass, where another summation order may round it to
# the other side of zero
TIE = 2.0 ** -21


class _Stop(Exception):
    def __init__(self, z):
        self.z = z


def _grad64(g, agent, rec, oracle, golden, adv_n):
    """The first minibatch's loss gradient in float64 on the CPU: the reference's CNNActorCritic (src/actor_critic.py:
    three convs + ReLU per tower, Linear(576, 512) + ReLU, the heads) and PPO loss (src/ppo.py:130-150) restated with
    F.conv2d / F.linear on the starting weights, the rendered frames, the given normalised advantages and returns.
    Returns (gradient per tensor, tie envelope per tensor): the envelope sums, over every ReLU unit whose pre-activation
    is a tie at fp32 precision (|z| <= TIE * its sum's absolute mass), the norm of that unit's gradient contribution
    (dL/dh at the unit times dz/dtheta for its sample) -- what a fp32 forward that rounds the tie to the other side
    adds or removes."""
    import torch.nn.functional as F

    B, MB, _ = (int(x) for x in g["cfg"])
    idx = torch.from_numpy(g["perms"][0][:MB])
    frames = torch.from_numpy(oracle.render(g["codes"], golden("atlas")["atlas"])).double()[idx]
    x_all = frames.permute(0, 3, 1, 2) / 255.0
    names = [n for n, _ in agent.ac.named_parameters()]
    P = {n: p.double().cpu().clone().requires_grad_(True) for n, p in zip(names, rec["p0"])}

    def net(x, stop=None):
        """(logits, values, [(key, z, h)]); with `stop`, raises _Stop(z) at that layer's pre-activation."""
        acts = []

        def relu(op, a, w, b, key, **kw):
            z = op(a, w, b, **kw)
            if key == stop:
                raise _Stop(z)
            with torch.no_grad():  # the sum's absolute mass, for the tie test
                mass = op(a.abs(), w.abs(), b.abs(), **kw)
            h = torch.relu(z)
            acts.append((key, z, h, mass))
            return h

        def tower(pre):
            w = lambda i: (P[f"{pre}.network.{i}.weight"], P[f"{pre}.network.{i}.bias"])  # noqa: E731
            h = relu(F.conv2d, x, *w(0), pre + ".0", stride=4)
            h = relu(F.conv2d, h, *w(2), pre + ".2", stride=2)
            h = relu(F.conv2d, h, *w(4), pre + ".4", stride=1)
            return h.flatten(1)

        ha = relu(F.linear, tower("actor_extractor"), P["actor.0.weight"], P["actor.0.bias"], "actor.0")
        hc = relu(F.linear, tower("critic_extractor"), P["critic.0.weight"], P["critic.0.bias"], "critic.0")
        logits = F.linear(ha, P["actor.2.weight"], P["actor.2.bias"])
        values = F.linear(hc, P["critic.2.weight"], P["critic.2.bias"]).squeeze(-1)
        return logits, values, acts

    logits, values, acts = net(x_all)
    lg = torch.log_softmax(logits, -1)
    act = torch.from_numpy(g["actions"])[idx]
    new_logp = lg.gather(1, act[:, None]).squeeze(1)
    entropy = -(lg.exp() * lg).sum(-1)
    old_logp = torch.from_numpy(g["logp"]).double()[idx]
    adv = adv_n.reshape(-1).double().cpu()[idx]
    ret = rec["ret"].reshape(-1).double().cpu()[idx]
    lr, gamma, lam, clip, vf, ent = (float(v) for v in g["hparams"])
    ratio = torch.exp(new_logp - old_logp)
    pi = -torch.min(ratio * adv, torch.clamp(ratio, 1 - clip, 1 + clip) * adv).mean()
    loss = pi + vf * ((values - ret) ** 2).mean() - ent * entropy.mean()
    outs = torch.autograd.grad(loss, list(P.values()) + [a[2] for a in acts])
    grads = list(outs[:len(P)])
    dh = {a[0]: d for a, d in zip(acts, outs[len(P):])}
    norm = torch.sqrt(sum((t ** 2).sum() for t in grads))
    coef = min(1.0, 0.5 / (float(norm) + 1e-6))
    env = [0.0] * len(grads)
    ties = 0
    for key, z, _, mass in acts:
        zz = z.detach()
        per = zz.numel() // zz.shape[0]
        for j in torch.nonzero((zz.abs() <= TIE * mass).reshape(-1)).reshape(-1).tolist():
            c = float(dh[key].reshape(-1)[j])
            if c == 0.0:
                continue
            ties += 1
            s = j // per  # the unit's sample
            try:
                net(x_all[s:s + 1], stop=key)
            except _Stop as e:
                zj = e.z.reshape(-1)[j % per]
            dz = torch.autograd.grad(zj, list(P.values()), allow_unused=True)
            for i, d in enumerate(dz):
                if d is not None:
                    env[i] += abs(c) * coef * float(d.norm())
    print(f"float64 reference: {ties} ReLU ties at fp32 precision (|z| <= 2^-21 of the sum's absolute mass)")
    return [t * coef for t in grads], env


def _run(golden, device, ref_adv=False):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO
    from test_gpu_obs_gae import pack

    g = golden("update_grad_ref")
    B, MB, EPOCHS = (int(x) for x in g["cfg"])
    lr, gamma, lam, clip, vf, ent = (float(x) for x in g["hparams"])
    env = MerlinVecEnv(1, "mediumhard", seed=1, device=device)
    perms = torch.from_numpy(g["perms"])
    torch.manual_seed(0)
    agent = PPO(env, lr=lr, gamma=gamma, lam=lam, clip_eps=clip, update_epochs=EPOCHS, batch_size=B,
                minibatch_size=MB, vf_coef=vf, ent_coef=ent, device=device, perm_fn=lambda n, e: perms[e])
    assert agent.conv1_from_codes and agent.dedup and agent.windows and agent.fast_step
    assert agent.ac.fc1_impl == "h3" and agent._clip_adam is not None
    for (k, t), (s, a, first) in zip(agent.ac.state_dict().items(), g["sums0"]):
        assert abs(t.double().sum().item() - s) <= 1e-5 * max(1.0, abs(a)), k  # the same init (up to LAPACK rounding)
    with torch.no_grad():  # the reference's exact starting weights (its orthogonal_ init ran on this container's CPU)
        for i, (_, p) in enumerate(agent.ac.named_parameters()):
            p.copy_(torch.from_numpy(g[f"p0_{i}"]).to(p.device))
    buf = agent.buf
    buf.codes[:B, 0] = torch.from_numpy(pack(g["codes"])).to(device)
    for dst, key, dt in ((buf.actions, "actions", torch.int64), (buf.logprobs, "logp", torch.float32),
                         (buf.values, "values", torch.float32), (buf.rewards, "rewards", torch.float32),
                         (buf.dones, "dones", torch.float32)):
        dst[:, 0] = torch.from_numpy(g[key]).to(device=device, dtype=dt)

    named = list(agent.ac.named_parameters())
    rec = {}
    step_orig = agent._clip_adam.step

    def step_wrap():
        first = "grads" not in rec
        if first:
            rec["p0"] = [p.detach().clone() for _, p in named]
            rec["grads"] = [p.grad.detach().clone() for _, p in named]
        norm = step_orig()
        if first:
            rec["norm"] = float(norm)
            rec["p1"] = [p.detach().clone() for _, p in named]
        return norm

    agent._clip_adam.step = step_wrap
    if ref_adv:  # the reference's normalisation (src/ppo.py:125, fp32 torch on the CPU) of the bit-exact GAE output
        adv_orig = agent._advantages

        def adv_wrap(rewards, values, dones, last_value, *a, **k):
            # the reference's own normalised advantages and returns, as its update computed them (stored in the
            # fixture: torch's fp32 CPU moments round by the host's vector ISA, so they are data, not recomputed)
            _, ret = adv_orig(rewards, values, dones, last_value, *a, **k)
            rec["adv_n"] = torch.from_numpy(g["adv_norm"]).to(ret.device).view_as(ret)
            ret.copy_(torch.from_numpy(g["returns"]).to(ret.device).view_as(ret))
            return rec["adv_n"], ret

        agent._advantages = adv_wrap
    stats = agent.update(float(g["last_value"]))
    rec.setdefault("adv_n", agent.last_adv_normalized)
    rec["ret"] = agent.buf.returns
    assert agent._wstep is not None  # the fast (benched) step ran, not the autograd fallback
    return g, agent, named, rec, stats, (B, MB, lr)


def _step_lr(rec, i, lr):
    return (rec["p1"][i].double() - rec["p0"][i].double()).cpu() / lr


def test_first_step_gradient_matches_reference(golden, oracle, device):
    """The reference's normalised advantages injected: gradient, pre-clip norm and first Adam step as the reference's;
    the epoch's statistics too."""
    g, agent, named, rec, stats, (B, MB, lr) = _run(golden, device, ref_adv=True)
    assert [n for n, _ in named] == [str(n) for n in g["param_names"]]
    assert agent.last_distinct_frac < 0.75  # the rollout repeats frames (0.52 distinct per sample): grouping exercised
    g64, env = _grad64(g, agent, rec, oracle, golden, rec["adv_n"])
    norm_ref = float(g["first_norm"])
    assert abs(rec["norm"] - norm_ref) <= 1e-5 * norm_ref, (rec["norm"], norm_ref)
    coef = min(1.0, 0.5 / (rec["norm"] + 1e-6))  # clip_grad_norm_'s coefficient (1 under the 0.5 norm)
    for i, (name, _) in enumerate(named):
        gr = torch.from_numpy(g[f"grad{i}"]).double()
        ours = rec["grads"][i].double().cpu() * coef
        d_ref, d64, d_ref64 = ((ours - gr).norm().item(), (ours - g64[i]).norm().item(), (gr - g64[i]).norm().item())
        n64 = g64[i].norm().item()
        print(f"{name:36s} |g| {n64:.3e}  ours vs reference {d_ref / n64:.2e}  vs float64: ours {d64 / n64:.2e}, "
              f"reference {d_ref64 / n64:.2e}  (tie envelope {env[i] / n64:.1e})")
        assert d_ref64 <= REL * n64 + env[i], (name, "the reference itself", d_ref64 / n64)
        assert d64 <= REL * n64 + env[i], (name, d64 / n64, env[i] / n64)
        assert d_ref <= 2 * REL * n64 + env[i], (name, d_ref / n64, env[i] / n64)
    # the first Adam step, lr units: g / (|g| + eps) per element -- where the reference gradient is clear of eps
    # (|g| >= 1e-6: a 1e-5 relative error in g moves the step by < 1e-5) it must match the reference's
    for i, (name, _) in enumerate(named):
        st_ref = torch.from_numpy(g[f"step{i}"].astype(np.float64))
        d = (_step_lr(rec, i, lr) - st_ref).abs()
        clear = torch.from_numpy(g[f"grad{i}"]).double().abs() >= 1e-6
        if clear.any():
            assert d[clear].max().item() <= 2e-3, (name, d[clear].max().item())  # (fp16-stored reference step)
        assert d.max().item() <= 2.0 + 1e-3, name  # anywhere: at most a sign flip of a ~eps gradient
    ref = dict(zip([str(k) for k in g["stat_names"]], g["stat_vals"]))
    for k, v in ref.items():  # the whole epoch's statistics (four optimizer steps)
        tol = 2.5 / MB if k == "clipfrac" else 2e-3 * max(1.0, abs(v))
        assert abs(stats[k] - v) <= tol, (k, stats[k], v)


def test_first_step_gradient_with_own_normalisation_matches_float64(golden, oracle, device):
    """The benched path as it runs (its f64-moment normalisation): every tensor within 1e-5 (+ the tie envelope) of
    the float64 gradient of its own advantages; the distance to the reference's gradient is printed."""
    g, agent, named, rec, stats, (B, MB, lr) = _run(golden, device)
    g64, env = _grad64(g, agent, rec, oracle, golden, rec["adv_n"])
    coef = min(1.0, 0.5 / (rec["norm"] + 1e-6))
    for i, (name, _) in enumerate(named):
        gr = torch.from_numpy(g[f"grad{i}"]).double()
        ours = rec["grads"][i].double().cpu() * coef
        n64 = g64[i].norm().item()
        d64 = (ours - g64[i]).norm().item()
        print(f"{name:36s} vs float64 {d64 / n64:.2e}  vs reference {((ours - gr).norm() / gr.norm()).item():.2e}  "
              f"(tie envelope {env[i] / n64:.1e})")
        assert d64 <= REL * n64 + env[i], (name, d64 / n64, env[i] / n64)
    ref = dict(zip([str(k) for k in g["stat_names"]], g["stat_vals"]))
    for k, v in ref.items():
        tol = 2.5 / MB if k == "clipfrac" else 2e-3 * max(1.0, abs(v))
        assert abs(stats[k] - v) <= tol, (k, stats[k], v)
