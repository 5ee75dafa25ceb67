"""GPU: the BENCHED update's gradient pinned to the reference's own gradient at a real minibatch size.

`update_grad_ref.npz` (tests/golden/make_golden.py gen_update_grad) holds the reference PPO.update
(src/ppo.py:122-168) on an 8,192-step single-env rollout of the C oracle's mediumhard env, one epoch of four
minibatches of 2,048, with the FIRST optimizer step recorded whole: every parameter's clipped gradient as
clip_grad_norm_ left it for Adam (:153-156), the pre-clip norm, and the parameters' change by that step.

Here the same inputs run through exactly what bench.py times -- code storage, the HIP GAE + normalisation, the
distinct-frame grouping, conv2 / conv3 once per receptive-field window, fc1's three GEMMs in h3 form over operand
planes (k_h3_pqg / k_h3_pq / k_h3_tq), the fused loss and the two-launch clip + Adam -- and the gradient the
benched path hands to its optimizer (p.grad at the first ClipAdam.step, clipped with the same coefficient) is
compared tensor by tensor: ||g - g_ref|| <= 1e-4 ||g_ref||.  The reference runs fp32 on the CPU, this path fp32
products on the GPU in other summation orders; 1e-4 is two orders above that noise and far below any
algorithmic difference (a dropped sample, a wrong window, a wrong tap moves a tensor by >= 1e-2).
The first Adam step is checked too: it is g / (|g| + eps) per element in units of lr, so it is held to the
reference's wherever the reference gradient is clear of eps."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REL = 1e-4  # per-tensor relative norm of the gradient difference


def _run(golden, device):
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
        assert abs(t.double().sum().item() - s) <= 1e-5 * max(1.0, abs(a)), k
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
        first = not rec
        if first:
            rec["p0"] = [p.detach().clone() for _, p in named]
            rec["grads"] = [p.grad.detach().clone() for _, p in named]
        norm = step_orig()
        if first:
            rec["norm"] = float(norm)
            rec["p1"] = [p.detach().clone() for _, p in named]
        return norm

    agent._clip_adam.step = step_wrap
    stats = agent.update(float(g["last_value"]))
    assert agent._wstep is not None  # the fast (benched) step ran, not the autograd fallback
    return g, agent, named, rec, stats, (B, MB, lr)


def test_first_step_gradient_matches_reference(golden, device):
    g, agent, named, rec, stats, (B, MB, lr) = _run(golden, device)
    assert [n for n, _ in named] == [str(n) for n in g["param_names"]]
    assert agent.last_distinct_frac < 0.75  # the rollout repeats frames (0.52 distinct per sample): grouping exercised
    # the pre-clip norm, and the coefficient clip_grad_norm_ applies (1 when the norm is under 0.5)
    norm_ref = float(g["first_norm"])
    assert abs(rec["norm"] - norm_ref) <= 1e-4 * norm_ref, (rec["norm"], norm_ref)
    coef = min(1.0, 0.5 / (rec["norm"] + 1e-6))
    worst = []
    for i, (name, _) in enumerate(named):
        gr = torch.from_numpy(g[f"grad{i}"]).double()
        ours = rec["grads"][i].double().cpu() * coef
        rel = ((ours - gr).norm() / gr.norm()).item()
        worst.append((rel, name))
        assert rel <= REL, (name, rel)
    print("per-tensor relative gradient error, worst:", sorted(worst)[-4:])
    # the first Adam step, lr units: g / (|g| + eps) per element -- where the reference gradient is clear of eps
    # (|g| >= 1e-6: a 1e-4 relative error in g moves the step by < 1e-6) it must match the reference's
    for i, (name, _) in enumerate(named):
        st_ref = torch.from_numpy(g[f"step{i}"].astype(np.float64))
        st = (rec["p1"][i].double() - rec["p0"][i].double()).cpu() / lr
        gr = torch.from_numpy(g[f"grad{i}"]).double().abs()
        clear = gr >= 1e-6
        d = (st - st_ref).abs()
        if clear.any():
            assert d[clear].max().item() <= 2e-3, (name, d[clear].max().item())
        assert d.max().item() <= 2.0 + 1e-3, name  # anywhere: at most a sign flip of a ~eps gradient
        if (d > 2e-3).any():
            print(f"{name}: {(d > 2e-3).float().mean().item():.2e} of the steps differ by > 2e-3 (|g_ref| < 1e-6 there)")
    # and the whole epoch's statistics (four optimizer steps)
    ref = dict(zip([str(k) for k in g["stat_names"]], g["stat_vals"]))
    for k, v in ref.items():
        tol = 2.5 / MB if k == "clipfrac" else 2e-3 * max(1.0, abs(v))
        assert abs(stats[k] - v) <= tol, (k, stats[k], v)
