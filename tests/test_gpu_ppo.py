"""GPU: the PPO update against the reference's own PPO.update (update_ref.npz),
replaying its randperm draws; plus an end-to-end vectorised iteration."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_update_matches_reference(golden, oracle, device):
    from merlin.ppo import PPO

    g = golden("update_ref")
    B, MB, EPOCHS = (int(x) for x in g["cfg"])
    lr, gamma, lam, clip, vf, ent = (float(x) for x in g["hparams"])
    frames = oracle.render(g["codes"], golden("atlas")["atlas"])

    class ReplayEnv:  # generic gym env path of PPO (f32 frame storage, as the reference)
        action_space = type("S", (), {"n": 3})()

        def reset(self, seed=None):
            return frames[0].copy(), {}

    torch.manual_seed(0)
    perms = torch.from_numpy(g["perms"])
    agent = PPO(ReplayEnv(), lr=lr, gamma=gamma, lam=lam, clip_eps=clip, update_epochs=EPOCHS, batch_size=B,
                minibatch_size=MB, vf_coef=vf, ent_coef=ent, device=device,
                perm_fn=lambda n, e: perms[e])
    sd = agent.ac.state_dict()
    # orthogonal_ init runs a CPU QR: another host's LAPACK may differ in the last bits
    for (k, t), (s, a, first) in zip(sd.items(), g["sums0"]):
        assert abs(t.double().sum().item() - s) <= 1e-5 * max(1.0, abs(a)), k
    for t in range(B):
        agent.buffer.add(torch.from_numpy(frames[t].astype(np.float32)).to(device),
                         torch.tensor(int(g["actions"][t])), torch.tensor(float(g["logp"][t])),
                         torch.tensor(float(g["values"][t])), torch.tensor(float(g["rewards"][t])),
                         torch.tensor(float(g["dones"][t])))
    stats = agent.update(float(g["last_value"]))
    ref = dict(zip([str(k) for k in g["stat_names"]], g["stat_vals"]))
    # reference on CPU vs MIOpen/rocBLAS on the GPU: ~1e-6 per-op differences; after 8 Adam
    # steps the averaged metrics agree to ~1e-4 relative
    for k, v in ref.items():
        assert abs(stats[k] - v) <= 2e-3 * max(1.0, abs(v)), (k, stats[k], v)
    # post-Adam parameters: an element whose gradient is ~0 (conv1 has many, behind dead
    # ReLUs) can take the opposite Adam step (+-lr per optimizer step) on CPU vs GPU; bound the
    # signed sum by the trajectories of up to 0.5% of the elements (at least 4) flipping
    nsteps = EPOCHS * ((B + MB - 1) // MB)
    for (k, t), (s, a, first) in zip(agent.ac.state_dict().items(), g["sums1"]):
        t = t.double().cpu()
        flips = max(4.0, 0.005 * t.numel())
        allow = 2 * lr * nsteps * flips
        assert abs(t.sum().item() - s) <= 1e-5 * a + allow, k
        assert abs(t.abs().sum().item() - a) <= 1e-5 * a + allow, k


def test_code_path_sgd_matches_frame_path(golden, oracle, device):
    """The vectorised path's minibatch SGD (HIP expansion of 32-B codes by index,
    /255 folded into the expansion) == the frame-storage path (f32 NHWC frames,
    permute + /255 in the model) on identical transitions, advantages and perms."""
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO
    from test_gpu_obs_gae import pack

    g = golden("update_ref")
    B, MB, EPOCHS = (int(x) for x in g["cfg"])
    frames = torch.from_numpy(oracle.render(g["codes"], golden("atlas")["atlas"]).astype(np.float32)).to(device)
    codes = torch.from_numpy(pack(g["codes"])).to(device)
    perms = torch.from_numpy(g["perms"])
    t = lambda k, dt=torch.float32: torch.from_numpy(g[k]).to(device=device, dtype=dt)  # noqa: E731
    rs = np.random.RandomState(4)
    adv = torch.from_numpy(rs.randn(B).astype(np.float32)).to(device)
    ret = torch.from_numpy(rs.randn(B).astype(np.float32)).to(device)
    results = []
    for use_codes in (True, False):
        env = MerlinVecEnv(B, "mediumhard", seed=1, device=device)
        torch.manual_seed(0)
        agent = PPO(env, batch_size=B, minibatch_size=MB, update_epochs=EPOCHS, ent_coef=0.05, device=device,
                    perm_fn=lambda n, e: perms[e])
        if use_codes:
            stats = agent._sgd(B, codes, None, t("actions", torch.int64), t("logp"), adv, ret)
        else:
            stats = agent._sgd(B, None, frames, t("actions", torch.int64), t("logp"), adv, ret)
        results.append((stats, [p.detach().clone() for p in agent.ac.parameters()]))
    (s1, p1), (s2, p2) = results
    for k in s1:
        assert abs(s1[k] - s2[k]) <= 1e-5 * max(1.0, abs(s2[k])), k
    # 8 Adam steps: Adam's m/sqrt(v) can flip a near-zero element's step (+-lr), so compare
    # each tensor by relative norm and bound the element error by a few lr=3e-4 steps' noise
    # 8 Adam steps amplify fp32 regrouping noise on near-zero-gradient elements (m/sqrt(v)
    # ~ +-1): a loose bound here, the exact comparison is the single-step gradient below
    for a, b in zip(p1, p2):
        d = (a - b).abs()
        assert d.max().item() <= 2 * 3e-4 * 8  # never more than every step flipped (lr 3e-4, 8 steps)
        assert (d > 5e-5).float().mean().item() < 0.05  # the bulk tracks closely
    # one minibatch, same weights: outputs and every parameter gradient
    from merlin.dedup import FrameGroups

    ac = agent.ac
    codes = agent.buf.flat_codes
    mb = torch.randperm(codes.shape[0], device=device)[:4096]
    acts = agent.buf.actions.reshape(-1)[mb]
    grads = []
    for grp in (FrameGroups(codes).minibatch(mb), None):
        ac.zero_grad()
        lp, ent, v = ac.evaluate_codes(codes, acts, index=mb, groups=grp)
        (-(lp.exp() * 0.3).mean() + 0.5 * (v ** 2).mean() - 0.05 * ent.mean()).backward()
        grads.append(([x.detach() for x in (lp, ent, v)], [p.grad.clone() for p in ac.parameters()]))
    (o1, g1), (o2, g2) = grads
    for a, b in zip(o1, o2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    for (name, _), a, b in zip(ac.named_parameters(), g1, g2):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 1e-5, name
        assert (a - b).abs().max().item() < 3e-5


def test_end_to_end_iteration(device):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    N, T = 512, 16
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=device, max_steps=12)
    torch.manual_seed(0)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, update_epochs=2, ent_coef=0.05, device=device)
    lv = agent.collect_rollouts()
    assert lv.shape == (N,)
    assert (agent.buf.dones.sum(0) >= 1).all()  # max_steps=12 < T: every env truncated at least once
    assert len(agent.episode_returns) == int(agent.buf.dones.sum().item())
    p0 = [p.detach().clone() for p in agent.ac.parameters()]
    stats = agent.update(lv)
    assert set(stats) == {"pi_loss", "v_loss", "entropy", "kl", "clipfrac", "gradnorm"}
    assert all(np.isfinite(v) for v in stats.values())
    assert any(not torch.equal(a, b) for a, b in zip(p0, agent.ac.parameters()))
    # the rollout observations are the env's: codes row t+1 = obs after action t
    assert agent.buf.codes.abs().sum() > 0


def test_dedup_update_matches_per_sample(device):
    """Distinct-frame grouping (merlin/dedup.py) leaves the update unchanged: same metrics and
    parameters (fp32 regrouping only) as evaluating the towers on every sample, on a real
    rollout (which revisits views)."""
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    N, T = 256, 32
    res = []
    for dedup in (True, False):
        env = MerlinVecEnv(N, "mediumhard", seed=777, device=device)
        torch.manual_seed(3)
        g = torch.Generator(device=device)
        g.manual_seed(11)
        agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=2, ent_coef=0.05,
                    device=device, dedup=dedup, perm_fn=lambda n, e: torch.randperm(n, device=device, generator=g))
        torch.manual_seed(4)
        lv = agent.collect_rollouts()
        stats = agent.update(lv)
        res.append((stats, [p.detach().clone() for p in agent.ac.parameters()], agent.last_distinct_frac))
    (s1, p1, frac), (s2, p2, none) = res
    assert none is None and 0.0 < frac < 1.0, frac  # the rollout does repeat observations
    for k in s1:
        # clipfrac counts samples past |ratio - 1| > clip: a ratio within fp32 noise of the
        # boundary may fall on either side (a few samples of a minibatch of 2048)
        tol = 4.0 / (N * T // 4) if k == "clipfrac" else 1e-4 * max(1.0, abs(s2[k]))
        assert abs(s1[k] - s2[k]) <= tol, (k, s1[k], s2[k])
    # 8 Adam steps amplify fp32 regrouping noise on near-zero-gradient elements (m/sqrt(v)
    # ~ +-1): a loose bound here, the exact comparison is the single-step gradient below
    for a, b in zip(p1, p2):
        d = (a - b).abs()
        assert d.max().item() <= 2 * 3e-4 * 8  # never more than every step flipped (lr 3e-4, 8 steps)
        assert (d > 5e-5).float().mean().item() < 0.05  # the bulk tracks closely
    # one minibatch, same weights: outputs and every parameter gradient
    from merlin.dedup import FrameGroups

    ac = agent.ac
    codes = agent.buf.flat_codes
    mb = torch.randperm(codes.shape[0], device=device)[:4096]
    acts = agent.buf.actions.reshape(-1)[mb]
    grads = []
    for grp in (FrameGroups(codes).minibatch(mb), None):
        ac.zero_grad()
        lp, ent, v = ac.evaluate_codes(codes, acts, index=mb, groups=grp)
        (-(lp.exp() * 0.3).mean() + 0.5 * (v ** 2).mean() - 0.05 * ent.mean()).backward()
        grads.append(([x.detach() for x in (lp, ent, v)], [p.grad.clone() for p in ac.parameters()]))
    (o1, g1), (o2, g2) = grads
    for a, b in zip(o1, o2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    for (name, _), a, b in zip(ac.named_parameters(), g1, g2):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 1e-5, name
