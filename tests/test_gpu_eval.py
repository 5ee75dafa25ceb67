"""GPU: batched deterministic evaluation (merlin/evaluation.py) against the C oracle: the episodes'
recorded actions replayed through oracle.batch_rollout (the same seeds: ppo/ppo_train.py:48
reset(seed=base + ep)) give the same first-done step and the same episode reward; and the
checkpoint sweep (src/sweep_checkpoints.py:72-100) ranks checkpoints on the fixed seeds."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("difficulty,max_steps", [("mediumhard", 40), ("easy", 60), ("mediumhard", None)])
def test_eval_matches_oracle_replay(oracle, device, difficulty, max_steps):
    from merlin.actor_critic import CNNActorCritic
    from merlin.evaluation import evaluate_seeds

    torch.manual_seed(7)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    seeds = list(range(1999, 1999 + 24))
    rew, steps, acts = evaluate_seeds(ac, seeds, difficulty=difficulty, device=device, max_steps=max_steps,
                                      record=True)
    acts = acts.numpy()
    codes, orew, oterm, otrunc, _ = oracle.batch_rollout(np.array(seeds, dtype=np.uint64), acts,
                                                         difficulty=difficulty, max_steps=max_steps or 0)
    done = np.maximum(oterm, otrunc).astype(bool)
    for i in range(len(seeds)):
        first = int(np.argmax(done[:, i])) if done[:, i].any() else None
        assert first is not None, i  # every episode ended inside the recorded actions
        assert steps[i] == first + 1, (i, steps[i], first + 1)
        # the episode reward is its (only nonzero) terminal reward; oracle f32 vs the env's f64 sum
        assert abs(rew[i] - float(orew[: first + 1, i].astype(np.float64).sum())) <= 1e-6, i


def _zero_shot_serial(ac, env, seed, device):
    """One seeded deterministic episode and its loss, step by step through the gym-API env and the
    frame path of the model, with the GAE in Python floats -- the procedure of
    src/distribution_over_tasks.py:71-120 restated (the yardstick for the batched version)."""
    obs, _ = env.reset(seed=seed)
    frames, acts, rews, vals = [], [], [], []
    total, done = 0.0, False
    while not done:
        o = torch.as_tensor(np.asarray(obs, dtype=np.float32), device=device).unsqueeze(0)
        with torch.no_grad():
            a, _, v = ac.act(o, deterministic=True)
        obs, r, term, trunc, _ = env.step(int(a.item()))
        done = term or trunc
        frames.append(o[0])
        acts.append(int(a.item()))
        rews.append(float(r))
        vals.append(float(v.item()))
        total += float(r)
    T = len(rews)
    adv, g = [0.0] * T, 0.0
    for t in reversed(range(T)):
        m = 0.0 if t == T - 1 else 1.0  # the value after the last step never enters
        nv = 0.0 if t == T - 1 else vals[t + 1]
        g = rews[t] + 0.995 * nv * m - vals[t] + 0.995 * 0.95 * m * g
        adv[t] = g
    adv = torch.tensor(adv, dtype=torch.float32, device=device)
    adv = (adv - adv.mean()) / (adv.std() + 1e-8) if T > 1 else torch.zeros_like(adv)
    ret = torch.tensor(vals, dtype=torch.float32, device=device) + adv
    with torch.no_grad():
        lp, _, nv = ac.evaluate(torch.stack(frames), torch.tensor(acts, device=device))
    loss = (-lp.mean() + 0.5 * ((nv - ret) ** 2).mean()).item()
    return total, T, loss


def test_zero_shot_matches_serial_episodes(device):
    """evaluate_zero_shot (all seeds at once, codes path, HIP GAE) == the serial restatement of
    src/distribution_over_tasks.py:71-120 (gym env, frame path): rewards and lengths exactly, the
    loss within fp32 summation noise."""
    from merlin import MerlinEnv
    from merlin.actor_critic import CNNActorCritic
    from merlin.evaluation import evaluate_seeds, evaluate_zero_shot

    torch.manual_seed(11)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    seeds = list(range(5000, 5010))
    rew, steps, loss = evaluate_zero_shot(ac, seeds, device=device, max_steps=48)
    r2, s2 = evaluate_seeds(ac, seeds, device=device, max_steps=48)
    assert rew == r2 and steps == s2
    env = MerlinEnv("mediumhard", device=device, max_steps=48)
    for i, sd in enumerate(seeds):
        tot, T, ls = _zero_shot_serial(ac, env, sd, device)
        assert T == steps[i] and abs(tot - rew[i]) <= 1e-6, (i, T, steps[i], tot, rew[i])
        assert abs(ls - loss[i]) <= 1e-4 * max(1.0, abs(ls)), (i, ls, loss[i])
    env.close()


def test_sweep_ranks_checkpoints(device, tmp_path):
    from merlin.actor_critic import CNNActorCritic
    from merlin.evaluation import SWEEP_SEED_BASE, evaluate_seeds, sweep_checkpoints

    for k in range(3):
        torch.manual_seed(100 + k)
        torch.save(CNNActorCritic((56, 56, 3), 3).state_dict(), tmp_path / f"ppo_model_{k}k.pth")
    res = sweep_checkpoints(str(tmp_path), "mediumhard", tasks=12, device=device, max_steps=64)
    assert len(res) == 3 and [r[1] for r in res] == sorted((r[1] for r in res), reverse=True)
    path, r0, s0 = res[0]
    from merlin.checkpoints import load_policy

    rew, steps = evaluate_seeds(load_policy(path, device), range(SWEEP_SEED_BASE, SWEEP_SEED_BASE + 12),
                                device=device, max_steps=64)
    assert abs(r0 - np.mean(rew)) < 1e-12 and abs(s0 - np.mean(steps)) < 1e-12
