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
