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
    for a, b in zip(p1, p2):
        assert ((a - b).norm() / b.norm()).item() < 1e-5
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
