"""GPU: the BENCHED update path pinned directly to the reference's own PPO.update (src/ppo.py:122-168).

The fixtures hold the reference's inputs (observation codes, actions, old log-probs, values, rewards,
dones, last value), its recorded randperm draws, and its outputs (the six update metrics and per-tensor
checksums of the post-Adam parameters):
  update_ref.npz          64 random frames, 2 epochs x 4 minibatches of 16
  update_rollout_ref.npz  a real 1,024-step single-env rollout of the C oracle's mediumhard env (440
                          distinct frames, 22 episode ends), 3 epochs x 4 minibatches of 256
Here they run through exactly what bench.py times: the vectorised code-storage path (MerlinVecEnv
storage layout [T][N]), GAE + normalisation on the HIP kernels, the distinct-frame grouping
(merlin/dedup.py), conv2 / conv3 once per receptive-field window (merlin/windows.py), fc1's three
GEMMs on the f16 matrix cores in two-plane form (h3: k_h3_ntpg / k_h3_ntp / k_h3_tng), the fused loss
(merlin_ppo_loss) and clip_grad_norm_ + Adam as two HIP launches (merlin_clip_adam).
Tolerances as tests/test_gpu_ppo.py::test_update_matches_reference (reference on CPU vs fp32 on the
GPU: ~1e-6 per-op differences; after the Adam steps metrics agree to ~1e-4 relative)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run_benched(golden, device, name):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO
    from test_gpu_obs_gae import pack

    g = golden(name)
    B, MB, EPOCHS = (int(x) for x in g["cfg"])
    lr, gamma, lam, clip, vf, ent = (float(x) for x in g["hparams"])
    env = MerlinVecEnv(1, "mediumhard", seed=1, device=device)  # N = 1: GAE over the B steps in order
    perms = torch.from_numpy(g["perms"])
    torch.manual_seed(0)
    agent = PPO(env, lr=lr, gamma=gamma, lam=lam, clip_eps=clip, update_epochs=EPOCHS, batch_size=B,
                minibatch_size=MB, vf_coef=vf, ent_coef=ent, device=device, perm_fn=lambda n, e: perms[e])
    # the benched configuration, not a fallback
    assert agent.conv1_from_codes and agent.dedup and agent.windows
    assert agent.ac.fc1_impl == "h3" and agent._clip_adam is not None  # the benched fc1 GEMMs (merlin_h3.hip)
    for (k, t), (s, a, first) in zip(agent.ac.state_dict().items(), g["sums0"]):
        assert abs(t.double().sum().item() - s) <= 1e-5 * max(1.0, abs(a)), k
    buf = agent.buf
    assert (buf.T, buf.N) == (B, 1)
    buf.codes[:B, 0] = torch.from_numpy(pack(g["codes"])).to(device)
    for dst, key, dt in ((buf.actions, "actions", torch.int64), (buf.logprobs, "logp", torch.float32),
                         (buf.values, "values", torch.float32), (buf.rewards, "rewards", torch.float32),
                         (buf.dones, "dones", torch.float32)):
        dst[:, 0] = torch.from_numpy(g[key]).to(device=device, dtype=dt)
    stats = agent.update(float(g["last_value"]))
    return g, agent, stats, (B, MB, EPOCHS, lr)


@pytest.mark.parametrize("name", ["update_ref", "update_rollout_ref"])
def test_benched_update_matches_reference(golden, device, name):
    g, agent, stats, (B, MB, EPOCHS, lr) = _run_benched(golden, device, name)
    assert agent.last_num_windows is not None and agent.last_num_windows > 0
    n_distinct = len(np.unique(g["codes"], axis=0))
    if name == "update_rollout_ref":
        assert n_distinct < B  # the rollout repeats observations: the grouping is exercised
    assert agent.last_distinct_frac is not None and agent.last_distinct_frac <= 1.0
    ref = dict(zip([str(k) for k in g["stat_names"]], g["stat_vals"]))
    for k, v in ref.items():
        # clipfrac is a count over the minibatch: a ratio within fp32 noise of 1 +- clip may fall on
        # either side (at most a couple of samples per minibatch over the update)
        tol = 2.5 / MB if k == "clipfrac" else 2e-3 * max(1.0, abs(v))
        assert abs(stats[k] - v) <= tol, (k, stats[k], v)
    # post-Adam parameters: elements with a ~0 gradient can take the opposite Adam step (+-lr per
    # optimizer step) on CPU vs GPU; bound the signed / absolute sums by the trajectories of up to
    # 0.5 % of a tensor's elements (at least 4) flipping on every step
    nsteps = EPOCHS * ((B + MB - 1) // MB)
    for (k, t), (s, a, first) in zip(agent.ac.state_dict().items(), g["sums1"]):
        t = t.double().cpu()
        allow = 2 * lr * nsteps * max(4.0, 0.005 * t.numel())
        assert abs(t.sum().item() - s) <= 1e-5 * a + allow, k
        assert abs(t.abs().sum().item() - a) <= 1e-5 * a + allow, k


def test_benched_update_tracks_frame_path_closely(golden, oracle, device):
    """The rollout fixture through the benched path and through the frame path (f32 NHWC frames
    rendered by the oracle, F.conv2d towers, the torch loss; same optimizer step): parameters after the
    whole update agree far inside the reference bound above, i.e. the benched path's distance to the
    reference is the fp32-on-GPU noise both share, not a property of the windows / x6 / fused kernels.
    The benched path is also bitwise deterministic run to run (fixed-order sums, no atomics)."""
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    g, agent, _, (B, MB, EPOCHS, lr) = _run_benched(golden, device, "update_rollout_ref")
    p1 = [p.detach().clone() for p in agent.ac.parameters()]
    _, agent2, _, _ = _run_benched(golden, device, "update_rollout_ref")
    for a, b in zip(p1, agent2.ac.parameters()):
        assert torch.equal(a, b.detach())
    env = MerlinVecEnv(1, "mediumhard", seed=1, device=device)
    perms = torch.from_numpy(g["perms"])
    torch.manual_seed(0)
    agent3 = PPO(env, lr=lr, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=EPOCHS, batch_size=B,
                 minibatch_size=MB, vf_coef=0.5, ent_coef=0.05, device=device, perm_fn=lambda n, e: perms[e],
                 conv1_from_codes=False)
    t = lambda k, dt=torch.float32: torch.from_numpy(g[k]).to(device=device, dtype=dt)  # noqa: E731
    adv, ret = agent3._advantages(t("rewards")[:, None].contiguous(), t("values")[:, None].contiguous(),
                                  t("dones")[:, None].contiguous(), torch.tensor([float(g["last_value"])], device=device))
    frames = torch.from_numpy(oracle.render(g["codes"], golden("atlas")["atlas"]).astype(np.float32)).to(device)
    agent3._sgd(B, None, frames, t("actions", torch.int64), t("logp"), adv.reshape(B), ret.reshape(B))
    p3 = [p.detach() for p in agent3.ac.parameters()]
    nsteps = EPOCHS * (B // MB)
    ds = [(a - b).abs().flatten() for a, b in zip(p1, p3)]
    for d in ds:
        assert d.max().item() <= 2 * lr * nsteps
    assert (torch.cat(ds) > 5e-5).float().mean().item() < 0.02
