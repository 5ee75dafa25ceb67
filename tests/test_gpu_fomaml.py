"""GPU: batched FOMAML (merlin.fomaml) vs a serial restatement of src/fomaml.py:110-212
replaying the same recorded support/query trajectories; and the reset-to-task-seed env."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_reseed_each_reset_replays_the_task_map(oracle, device):
    from merlin import MerlinVecEnv

    seeds = np.array([5, 77, 1234, 99999], dtype=np.uint64)
    env = MerlinVecEnv(4, "mediumhard", device=device, seeds=seeds, reseed_each_reset=True, max_steps=7)
    env.reset()
    st0 = env.get_state()
    for i, s in enumerate(seeds):
        cells, meta = oracle.gen_map(16, "mediumhard", int(s))
        assert (st0["cells"][i] == cells).all() and tuple(st0["agent_pos"][i]) == tuple(meta[:2])
    acts = torch.full((4,), 2, dtype=torch.int64, device=device)
    for _ in range(7 * 3):  # three truncated episodes, auto-reset each time
        env.step_into(acts)
    st = env.get_state()
    assert (st["walls"] == st0["walls"]).all()
    assert (st["agent_pos"] == st0["agent_pos"]).all() and (st["agent_dir"] == st0["agent_dir"]).all()


def _serial_loss(model, batch, g, gamma=0.995, lam=0.95):
    """compute_loss (src/fomaml.py:110-156) for task g on the recorded batch."""
    from merlin import _native as nat

    rews = batch["rew"][:, g].cpu().numpy()
    vals = batch["val"][:, g].cpu().numpy()
    dones = batch["done"][:, g].cpu().numpy()
    last_val = float(batch["last_val"][g].item())
    adv = np.zeros_like(rews)
    gae = 0.0
    for t in reversed(range(len(rews))):
        mask = 1.0 - dones[t]
        next_v = last_val if t == len(rews) - 1 else vals[t + 1]
        delta = rews[t] + gamma * next_v * mask - vals[t]
        gae = delta + gamma * lam * mask * gae
        adv[t] = gae
    dev = batch["rew"].device
    adv_t = torch.tensor(adv, dtype=torch.float32, device=dev)
    adv_t = (adv_t - adv_t.mean()) / (adv_t.std() + 1e-8)
    ret_t = (batch["val"][:, g] + adv_t).detach()
    k = len(rews)
    frames = nat.expand_obs(batch["codes"][:k, g].contiguous(), scale=1.0 / 255.0)
    new_logp, entropy, new_vals = model.evaluate(frames, batch["act"][:, g], prescaled=True)
    ratio = torch.exp(new_logp - batch["logp"][:, g])
    surr1 = ratio * adv_t
    surr2 = torch.clamp(ratio, 0.8, 1.2) * adv_t
    return -torch.min(surr1, surr2).mean() + 0.5 * ((new_vals - ret_t) ** 2).mean() - 0.05 * entropy.mean()


def test_meta_step_matches_serial_reference(device):
    from merlin import ScenarioCreator
    from merlin.fomaml import FOMAML

    torch.manual_seed(0)
    fm = FOMAML(ScenarioCreator(), lr_inner=0.01, lr_outer=3e-4, device=device, difficulty="mediumhard")
    meta0 = copy.deepcopy(fm.meta_policy)
    recorded = []
    orig = fm.collect_trajectory

    def rec(env, params, steps):
        b = orig(env, params, steps)
        recorded.append(b)
        return b

    fm.collect_trajectory = rec
    seeds = [11, 2024, 31337, 7]
    avg_loss, avg_rew, avg_steps, stats = fm.meta_train_step(seeds, k_support=48, k_query=48)
    support, query = recorded
    # serial restatement of meta_train_step on the recorded trajectories
    meta = copy.deepcopy(meta0)
    grads = [torch.zeros_like(p) for p in meta.parameters()]
    qlosses = []
    for g in range(len(seeds)):
        fast = copy.deepcopy(meta0)
        opt = torch.optim.SGD(fast.parameters(), lr=0.01)
        loss = _serial_loss(fast, support, g)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(fast.parameters(), max_norm=0.5)
        opt.step()
        ql = _serial_loss(fast, query, g)
        fast.zero_grad()
        ql.backward()
        for acc, p in zip(grads, fast.parameters()):
            acc += p.grad
        qlosses.append(ql.item())
    for p, g in zip(meta.parameters(), grads):
        p.grad = g / len(seeds)
    torch.nn.utils.clip_grad_norm_(meta.parameters(), max_norm=0.5)
    torch.optim.Adam(meta.parameters(), lr=3e-4).step()
    assert abs(avg_loss - float(np.mean(qlosses))) <= 1e-4 * max(1.0, abs(avg_loss))
    # the clipped meta gradients (left in .grad by both) agree to fp32 tolerance; the Adam
    # step itself (lr * g / |g| for a first step) can differ by sign where a gradient is
    # exactly 0 on one path (dead ReLU) and +-1e-12 on the other, so bound it by 2*lr
    gnorm = torch.sqrt(sum((p.grad ** 2).sum() for p in meta.parameters())).item()
    for (n, a), b in zip(fm.meta_policy.named_parameters(), meta.parameters()):
        # tensors whose gradient is itself a near-cancellation (the value-head bias: mean of
        # new_vals - vals - normalised adv) are judged against the global gradient norm
        scale = max(b.grad.norm().item(), 1e-3 * gnorm)
        rel = ((a.grad - b.grad).norm().item()) / scale
        assert rel < 1e-4, (n, rel)
        assert (a - b).abs().max().item() <= 2 * 3e-4 + 1e-6, n
