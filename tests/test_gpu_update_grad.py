"""GPU: the BENCHED update's gradient pinned to the reference's own gradient at a real minibatch size.

`update_grad_ref.npz` (tests/golden/make_golden.py gen_update_grad) holds the reference PPO.update
(src/ppo.py:122-168) on an 8,192-step single-env rollout of the C oracle's mediumhard env, one epoch of four
minibatches of 2,048, with the FIRST optimizer step recorded whole: every parameter's clipped gradient as
clip_grad_norm_ left it for Adam (:153-156), the pre-clip norm, and the parameters' change by that step.

Here the same inputs run through exactly what bench.py times -- code storage, the HIP GAE, the distinct-frame
grouping, conv2 / conv3 once per receptive-field window, fc1's three GEMMs in h3 form over operand planes (k_h3_pqg /
k_h3_pq / k_h3_tq), the fused loss and the two-launch clip + Adam -- and the gradient the benched path hands to its
optimizer (p.grad at the first ClipAdam.step) is compared tensor by tensor with the reference's and with the same
gradient in float64 (the reference's network and loss restated below on the CPU in double).

The starting weights are the reference's, loaded from the fixture (torch's orthogonal_ init goes through the host's
LAPACK, whose rounding differs between CPUs; at these weights the actor tower's gradient is a near-cancelling sum
that turns a 1e-7 weight difference into ~6e-4 of gradient).  One input differs by design: the reference normalises the advantages with fp32 torch moments (src/ppo.py:125), the
benched path with f64 moments (k_gae_thread + k_adv_normalize; the GAE itself is bit-exact).  At the initial weights
the actor's gradient is a near-cancelling sum (|g| ~ 1e-5 per weight): a ~1e-8 shift of the normalised advantages
moves it by ~6e-4 relative.  So the test runs the update twice:
  * with the reference's normalised advantages and returns injected (recorded by the generator from the reference's
    own compute_gae and fp32 moments):
    ||g - g_ref|| <= 1e-5 ||g_ref|| for every tensor, and the first Adam step equal wherever |g_ref| >= 1e-6;
  * with the benched path's own normalisation: every tensor within 1e-5 of the float64 gradient of ITS advantages
    (the reference's own fp32 gradient is within ~2.5e-6 of float64 on its advantages)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REL = 1e-5  # per-tensor relative norm of the gradient difference


def _grad64(g, agent, rec, oracle, golden, adv_n):
    """The first minibatch's loss gradient in float64 on the CPU: the reference's CNNActorCritic (src/actor_critic.py:
    three convs + ReLU per tower, Linear(576, 512) + ReLU, the heads) and PPO loss (src/ppo.py:130-150) restated with
    F.conv2d / F.linear on the starting weights, the rendered frames, and the benched path's advantages / returns
    (bit-exact with the reference's, tests/test_gpu_obs_gae.py)."""
    import torch.nn.functional as F

    B, MB, _ = (int(x) for x in g["cfg"])
    idx = torch.from_numpy(g["perms"][0][:MB])
    frames = torch.from_numpy(oracle.render(g["codes"], golden("atlas")["atlas"])).double()[idx]
    x = frames.permute(0, 3, 1, 2) / 255.0
    P = {n: p.double().cpu().requires_grad_(True) for (n, _), p in zip(agent.ac.named_parameters(), rec["p0"])}

    def tower(pre):
        h = F.relu(F.conv2d(x, P[pre + ".network.0.weight"], P[pre + ".network.0.bias"], stride=4))
        h = F.relu(F.conv2d(h, P[pre + ".network.2.weight"], P[pre + ".network.2.bias"], stride=2))
        h = F.relu(F.conv2d(h, P[pre + ".network.4.weight"], P[pre + ".network.4.bias"], stride=1))
        return h.flatten(1)

    ha = F.relu(F.linear(tower("actor_extractor"), P["actor.0.weight"], P["actor.0.bias"]))
    logits = F.linear(ha, P["actor.2.weight"], P["actor.2.bias"])
    hc = F.relu(F.linear(tower("critic_extractor"), P["critic.0.weight"], P["critic.0.bias"]))
    values = F.linear(hc, P["critic.2.weight"], P["critic.2.bias"]).squeeze(-1)
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
    grads = torch.autograd.grad(loss, list(P.values()))
    norm = torch.sqrt(sum((t ** 2).sum() for t in grads))
    coef = min(1.0, 0.5 / (float(norm) + 1e-6))
    return [t * coef for t in grads]


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
    g64 = _grad64(g, agent, rec, oracle, golden, rec["adv_n"])
    norm_ref = float(g["first_norm"])
    assert abs(rec["norm"] - norm_ref) <= 1e-5 * norm_ref, (rec["norm"], norm_ref)
    coef = min(1.0, 0.5 / (rec["norm"] + 1e-6))  # clip_grad_norm_'s coefficient (1 under the 0.5 norm)
    for i, (name, _) in enumerate(named):
        gr = torch.from_numpy(g[f"grad{i}"]).double()
        ours = rec["grads"][i].double().cpu() * coef
        rel = ((ours - gr).norm() / gr.norm()).item()
        e_ours = ((ours - g64[i]).norm() / g64[i].norm()).item()
        e_ref = ((gr - g64[i]).norm() / g64[i].norm()).item()
        print(f"{name:36s} |g| {gr.norm().item():.3e}  vs reference {rel:.2e}  vs float64: ours {e_ours:.2e}, "
              f"reference {e_ref:.2e}")
        assert rel <= REL, (name, rel, e_ours, e_ref)
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
    """The benched path as it runs (its f64-moment normalisation): every tensor within 1e-5 of the float64 gradient
    of its own advantages; the distance to the reference's gradient is printed (the actor tower's ~6e-4 is the
    normalisation's, see the module docstring)."""
    g, agent, named, rec, stats, (B, MB, lr) = _run(golden, device)
    g64 = _grad64(g, agent, rec, oracle, golden, rec["adv_n"])
    coef = min(1.0, 0.5 / (rec["norm"] + 1e-6))
    for i, (name, _) in enumerate(named):
        gr = torch.from_numpy(g[f"grad{i}"]).double()
        ours = rec["grads"][i].double().cpu() * coef
        e_ours = ((ours - g64[i]).norm() / g64[i].norm()).item()
        print(f"{name:36s} vs float64 {e_ours:.2e}  vs reference {((ours - gr).norm() / gr.norm()).item():.2e}")
        assert e_ours <= REL, (name, e_ours)
    ref = dict(zip([str(k) for k in g["stat_names"]], g["stat_vals"]))
    for k, v in ref.items():
        tol = 2.5 / MB if k == "clipfrac" else 2e-3 * max(1.0, abs(v))
        assert abs(stats[k] - v) <= tol, (k, stats[k], v)
