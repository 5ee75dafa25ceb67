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

    def rec(env, params, steps, **kw):
        b = orig(env, params, steps, **kw)
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


def _fixture_batch(fx, tag, G, device):
    """The fixture's per-task batches as merlin.fomaml's [k][tasks] batch dict (codes packed)."""
    from test_windows import pack

    codes = np.stack([pack(fx[f"t{g}_{tag}_codes"]) for g in range(G)], 1)  # [k+1, G, 8]
    b = {"codes": torch.from_numpy(codes).to(device)}
    for k in ("act", "rew", "val", "logp", "done"):
        b[k] = torch.from_numpy(np.stack([fx[f"t{g}_{tag}_{k}"] for g in range(G)], 1)).to(device)
    b["last_val"] = torch.tensor([float(fx[f"t{g}_{tag}_last_val"]) for g in range(G)], device=device)
    return b


def test_loss_and_meta_gradient_match_reference_fixture(golden, device):
    """Pinned to the reference itself (tests/golden/fomaml_ref.npz, made by importing
    src/fomaml.py): per task, compute_loss (src/fomaml.py:110-156) on the recorded support batch,
    the clipped inner SGD step, compute_loss on the recorded query batch with the adapted weights,
    and the meta gradient sum/n_tasks (:158-209), all through merlin.fomaml's batched path (HIP GAE,
    stacked per-task weights).  Tolerances: fp32 sums in another order (losses 1e-5 relative,
    gradients 1e-4 of each parameter's norm)."""
    from merlin import ScenarioCreator
    from merlin import batched_policy as bp
    from merlin.fomaml import FOMAML

    fx = golden("fomaml_ref")
    G, K = (int(x) for x in fx["cfg"])
    torch.manual_seed(0)  # the reference's init order: the same weights (cnn_ref checks it)
    fm = FOMAML(ScenarioCreator(), lr_inner=float(fx["lr_inner"]), lr_outer=3e-4, device=device,
                difficulty="mediumhard")
    names = [n for n, _ in fm.meta_policy.named_parameters()]
    support, query = _fixture_batch(fx, "s", G, device), _fixture_batch(fx, "q", G, device)
    fast = bp.stack_params(fm.meta_policy, G)
    loss_s, st_s = fm.compute_loss(support, fast)
    keys = ("pi_loss", "v_loss", "entropy", "kl", "clipfrac")
    for g in range(G):
        assert abs(float(st_s["loss"][g]) - float(fx[f"t{g}_s_loss"])) <= 1e-5 * max(1.0, abs(float(fx[f"t{g}_s_loss"])))
        for j, k in enumerate(keys):
            assert abs(float(st_s[k][g]) - float(fx[f"t{g}_s_stats"][j])) <= 1e-5, (g, k)
    grads = dict(zip(names, torch.autograd.grad(loss_s, [fast[n] for n in names])))
    grads, _ = fm._clip_per_task(grads, 0.5)
    with torch.no_grad():
        adapted = {n: (fast[n] - fm.lr_inner * grads[n]).detach().requires_grad_(True) for n in names}
    loss_q, st_q = fm.compute_loss(query, adapted)
    for g in range(G):
        assert abs(float(st_q["loss"][g]) - float(fx[f"t{g}_q_loss"])) <= 1e-5 * max(1.0, abs(float(fx[f"t{g}_q_loss"])))
        for j, k in enumerate(keys):
            assert abs(float(st_q[k][g]) - float(fx[f"t{g}_q_stats"][j])) <= 1e-5, (g, k)
    qgrads = dict(zip(names, torch.autograd.grad(loss_q, [adapted[n] for n in names])))
    assert list(fx["grad_names"]) == names
    gnorm = float(np.sqrt((fx["grad_stats"][:, 0] ** 2).sum()))
    for i, n in enumerate(names):
        gm = (qgrads[n].sum(0) / G).reshape(-1).double().cpu()
        ref_norm = float(fx["grad_stats"][i, 0])
        scale = max(ref_norm, 1e-3 * gnorm)
        assert abs(gm.norm().item() - ref_norm) <= 1e-4 * scale, n
        sel = fx["grad_idx"][i]
        sel = sel[sel >= 0]
        err = (gm[torch.from_numpy(sel)] - torch.from_numpy(fx["grad_vals"][i][:sel.size])).abs().max().item()
        assert err <= 1e-4 * scale, (n, err, scale)


def test_meta_step_at_cfg5_size(device):
    """BASELINE cfg 5 at its stated size: 32 tasks x 256 support + 256 query steps through
    meta_train_step (batched rollouts, inner SGD, meta Adam): finite outputs, parameters move."""
    from merlin import ScenarioCreator
    from merlin.fomaml import FOMAML

    torch.manual_seed(1)
    fm = FOMAML(ScenarioCreator(), lr_inner=0.01, lr_outer=3e-4, device=device, difficulty="mediumhard")
    p0 = [p.detach().clone() for p in fm.meta_policy.parameters()]
    seeds = np.random.RandomState(42).choice(100000, 32, replace=False)
    avg_loss, avg_rew, avg_steps, stats = fm.meta_train_step(seeds, k_support=256, k_query=256)
    assert np.isfinite(avg_loss) and np.isfinite(avg_rew) and 0 < avg_steps <= 1024
    assert all(np.isfinite(v) for v in stats.values())
    moved = sum(int((a != b).any()) for a, b in zip(p0, fm.meta_policy.parameters()))
    assert moved == len(p0)
