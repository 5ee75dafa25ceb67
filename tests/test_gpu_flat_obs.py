"""GPU: the batched trainer on flattened observations (scenario.yaml observation.flatten, src/scenario_creator/
scenario_creator.py:45-53 -> the reference's MLPActorCritic path, src/ppo.py:38-41): MerlinVecEnv(flatten=True[,
fully_observable=True]) gives the wrapped observations of the single env, PPO steps N envs with the MLP (the act and
the loss are the reference's torch ops; env step, auto-reset, GAE on the HIP kernels), and the batched evaluation
drives an MLP policy."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("full", [False, True])
def test_vec_flat_obs_equals_single_env(device, full):
    from merlin import MerlinEnv, MerlinVecEnv

    seeds = list(range(5, 13))
    vec = MerlinVecEnv(len(seeds), "easy", device=device, seeds=seeds, flatten=True, fully_observable=full)
    codes = vec.reset()
    got = (vec.render_full().reshape(len(seeds), -1) if full else vec.flat_obs(codes)).cpu().numpy()
    D = 768 if full else 56 * 56 * 3
    assert vec.observation_space.shape == (D,) and got.shape == (len(seeds), D)
    for i, s in enumerate(seeds):
        one = MerlinEnv("easy", device=device, flatten=True, fully_observable=full)
        obs, _ = one.reset(seed=s)
        assert np.array_equal(got[i], obs.astype(np.float32)), s


@pytest.mark.parametrize("full", [False, True])
def test_batched_mlp_rollout_and_update(device, full):
    from merlin import MerlinVecEnv
    from merlin.actor_critic import MLPActorCritic
    from merlin.ppo import PPO

    N, T = 128, 16
    env = MerlinVecEnv(N, "mediumhard", seed=31, device=device, max_steps=12, flatten=True, fully_observable=full)
    mirror = MerlinVecEnv(N, "mediumhard", seed=31, device=device, max_steps=12)
    torch.manual_seed(0)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=2, ent_coef=0.05, device=device)
    assert isinstance(agent.ac, MLPActorCritic) and agent.obs_shape == ((768,) if full else (56 * 56 * 3,))
    buf = agent.buf
    for it in range(2):
        lv = agent.collect_rollouts()
        # the rollout is a valid trajectory: the recorded actions replayed through a plain env give its frames
        codes = torch.zeros_like(buf.codes)
        rew, done = torch.zeros_like(buf.rewards), torch.zeros_like(buf.dones)
        mirror.reset(out=codes[0])
        for t in range(T):
            if full:
                assert torch.equal(agent._full_obs[t], mirror.render_full().reshape(N, -1)), t
            mirror.step_into(buf.actions[t].contiguous(), codes[t + 1], rew[t], None, None, done[t])
        assert torch.equal(codes, buf.codes)
        assert torch.equal(rew, buf.rewards) and torch.equal(done, buf.dones)
        assert (done.sum(0) >= 1).all()  # max_steps 12 < T: every env auto-reset
        assert ((buf.actions >= 0) & (buf.actions < 3)).all()
        # the stored log-probs / values are the MLP's on the flattened observations
        with torch.no_grad():
            for t in (0, T - 1):
                x = agent._flat_obs_at(t)
                lp, _, v = agent.ac.evaluate(x, buf.actions[t])
                torch.testing.assert_close(lp, buf.logprobs[t], rtol=1e-5, atol=1e-5)
                torch.testing.assert_close(v, buf.values[t], rtol=1e-5, atol=1e-5)
            _, _, v = agent.ac.act(agent._flat_obs_at(T))
            torch.testing.assert_close(v, buf.last_value, rtol=1e-5, atol=1e-5)
        before = [p.detach().clone() for p in agent.ac.parameters()]
        stats = agent.update(lv)
        assert all(np.isfinite(v) for v in stats.values()), stats
        assert any(not torch.equal(a, p) for a, p in zip(before, agent.ac.parameters()))
    mirror.errors()


def test_minibatch_flat_obs_are_the_samples(device):
    """The update's minibatch observations (PPO._minibatch_obs) are the flattened frames of exactly the sampled
    (step, env) pairs, rebuilt from the stored tile codes."""
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    N, T = 128, 8
    env = MerlinVecEnv(N, "mediumhard", seed=7, device=device, flatten=True)
    torch.manual_seed(1)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 2, update_epochs=1, device=device)
    agent.collect_rollouts()
    idx = torch.randperm(N * T, device=device)[:300]
    obs, pre = agent._minibatch_obs(agent.buf.flat_codes, None, idx)
    want = torch.stack([env.flat_obs(agent.buf.codes[int(k) // N])[int(k) % N] for k in idx.tolist()])
    assert not pre and torch.equal(obs, want)


def test_scenario_creator_vec_observation_modes(device, tmp_path):
    from merlin.actor_critic import MLPActorCritic
    from merlin.ppo import PPO
    from merlin.scenario_creator import ScenarioCreator

    def cfg(full, flat):
        p = tmp_path / f"s{int(full)}{int(flat)}.yaml"
        p.write_text(f"observation:\n  fully_observable: {str(full).lower()}\n  flatten: {str(flat).lower()}\n"
                     "difficulties:\n  easy:\n    env_id: MERLIN-Easy-v0\n    params:\n      size: 16\n")
        return ScenarioCreator(str(p))

    env = cfg(True, True).create_vec_env("easy", 128, seed=3, device=device)
    assert env.flatten and env.fully_observable and env.observation_space.shape == (768,)
    agent = PPO(env, batch_size=128 * 4, minibatch_size=256, update_epochs=1, device=device)
    assert isinstance(agent.ac, MLPActorCritic)
    assert all(np.isfinite(v) for v in agent.update(agent.collect_rollouts()).values())
    env = cfg(False, True).create_vec_env("easy", 128, seed=3, device=device)
    assert env.observation_space.shape == (56 * 56 * 3,)
    with pytest.raises(ValueError):
        cfg(True, False).create_vec_env("easy", 128, seed=3, device=device)


@pytest.mark.parametrize("full", [False, True])
def test_batched_eval_of_mlp_matches_serial_single_env(device, full):
    """evaluate_policy with an MLP policy (ppo/ppo_train.py's per-iteration eval on a flatten config): the batched
    episodes equal the reference's serial loop on single envs (deterministic argmax actions)."""
    from merlin import MerlinEnv
    from merlin.actor_critic import MLPActorCritic
    from merlin.evaluation import evaluate_policy

    torch.manual_seed(2)
    D = 768 if full else 56 * 56 * 3
    ac = MLPActorCritic(D, 3).to(device)
    rew, steps = evaluate_policy(ac, "easy", episodes=4, seed=900, size=16, device=device, max_steps=40)
    for ep in range(4):
        env = MerlinEnv("easy", device=device, max_steps=40, flatten=True, fully_observable=full)
        obs, _ = env.reset(seed=900 + ep)
        total, n = 0.0, 0
        while True:
            with torch.no_grad():
                a, _, _ = ac.act(torch.as_tensor(obs, dtype=torch.float32, device=device).view(1, -1),
                                 deterministic=True)
            obs, r, term, trunc, _ = env.step(int(a.item()))
            total += r
            n += 1
            if term or trunc:
                break
        # (the single env returns each reward rounded to float32 like the reference's tensor; the batched return is
        # the env's f64 accumulator)
        assert n == steps[ep] and abs(total - rew[ep]) < 1e-6, (ep, n, steps[ep], total, rew[ep])
