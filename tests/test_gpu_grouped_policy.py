"""GPU: merlin.grouped_policy (one weight set per task on the tile-code path, FOMAML's batched policies)
against CNNActorCritic run task by task with that task's weights: forward outputs, every parameter's
gradient, and the acting path (one frame per task).  fp32 sums regrouped: rtol 1e-5 on outputs, 1e-4
of each tensor's norm on gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _tasks(device, G, seed=0):
    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(seed)
    models = []
    for g in range(G):
        m = CNNActorCritic((56, 56, 3), 3).to(device)
        with torch.no_grad():  # distinct weights per task, all within the init's scale
            for p in m.parameters():
                p.add_(torch.randn_like(p) * 0.05 * (p.abs().mean() + 1e-3))
        models.append(m)
    params = {n: torch.stack([dict(m.named_parameters())[n].detach() for m in models]).requires_grad_(True)
              for n, _ in models[0].named_parameters()}
    return models, params


def _codes(device, n, seed):
    from test_gpu_conv2lut import _codes as c

    return c(device, n, seed=seed)[1]


@pytest.mark.parametrize("G,F", [(3, 37), (2, 256), (5, 4)])
def test_grouped_evaluate_matches_per_task_models(device, G, F):
    from merlin import grouped_policy as gp

    models, params = _tasks(device, G, seed=G * 100 + F)
    codes = _codes(device, G * F, seed=F)
    acts = torch.randint(0, 3, (G, F), device=device)
    lp, ent, v = gp.evaluate(params, codes, F, acts)
    w = torch.randn(G, F, device=device)
    loss = ((lp.exp() * w).sum() + (v ** 2 * w).sum() - 0.05 * ent.sum())
    loss.backward()
    for g, m in enumerate(models):
        rows = codes[g * F:(g + 1) * F]
        lp2, ent2, v2 = m.evaluate_codes(rows, acts[g])
        torch.testing.assert_close(lp[g], lp2, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(ent[g], ent2, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(v[g], v2, rtol=1e-5, atol=1e-5)
        m.zero_grad()
        ((lp2.exp() * w[g]).sum() + (v2 ** 2 * w[g]).sum() - 0.05 * ent2.sum()).backward()
        for n, p in m.named_parameters():
            ref = p.grad
            got = params[n].grad[g]
            rel = ((got - ref).norm() / ref.norm().clamp_min(1e-12)).item()
            assert rel < 1e-4, (g, n, rel)


def test_grouped_act_packed_matches_per_task_models(device):
    from merlin import grouped_policy as gp

    G = 6
    models, params = _tasks(device, G, seed=9)
    codes = _codes(device, G, seed=4)
    pk = gp.pack({k: v.detach() for k, v in params.items()})
    a, lp, v = gp.act_packed(pk, codes, deterministic=True)
    for g, m in enumerate(models):
        with torch.no_grad():
            a2, lp2, v2 = m.act_codes(codes[g:g + 1], deterministic=True)
        assert int(a[g]) == int(a2[0])
        torch.testing.assert_close(lp[g], lp2[0], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(v[g], v2[0], rtol=1e-5, atol=1e-5)
    # sampled draws follow the policy's law: 400 draws per task vs its probabilities
    cnt = torch.zeros(G, 3, device=device)
    for _ in range(400):
        a, _, _ = gp.act_packed(pk, codes)
        cnt[torch.arange(G, device=device), a] += 1
    for g, m in enumerate(models):
        with torch.no_grad():
            lp3, _, _ = m.evaluate_codes(codes[g:g + 1].repeat(3, 1), torch.arange(3, device=device))
        p = lp3.exp()
        freq = cnt[g] / 400
        assert ((freq - p).abs() <= 5 * torch.sqrt(p * (1 - p) / 400) + 0.01).all(), (g, freq, p)


@pytest.mark.parametrize("G", [1, 6, 32])
def test_group_act_parts_match_per_task_models(device, G):
    """merlin_group_act (FOMAML's acting step in two launches, round 5): the head partials summed (biases folded into
    chunk 0) give each task's logits / value of its own model on its own frame; drawn deterministically through
    act_draw with zero biases they give that model's argmax action and log-prob."""
    from merlin import _native as nat
    from merlin import grouped_policy as gp

    models, params = _tasks(device, G, seed=13 + G)
    codes = _codes(device, G, seed=G)
    pk = gp.pack({k: v.detach() for k, v in params.items()})
    part = gp.act_parts(pk, codes)
    assert part.shape == (2, 8, G, 4)
    logits, value = part[0].sum(0)[:, :3], part[1].sum(0)[:, 0]
    zb = torch.zeros(4, device=device)
    a, lp, v = nat.act_draw(part.contiguous(), zb[:3], zb[:1], deterministic=True)
    for g, m in enumerate(models):
        with torch.no_grad():
            lg, vv = m._forward_codes(codes[g:g + 1], None)
            a2, lp2, v2 = m.act_codes(codes[g:g + 1], deterministic=True)
        torch.testing.assert_close(logits[g], lg[0], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(value[g], vv[0], rtol=1e-5, atol=1e-5)
        assert int(a[g]) == int(a2[0])
        torch.testing.assert_close(lp[g], lp2[0], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(v[g], v2[0], rtol=1e-5, atol=1e-5)


def test_group_act_shared_weights_equal_per_task_copies(device):
    """merlin_group_act with ONE weight set for every task (shared_weights: FOMAML's support rollout, where each fast
    policy is still the meta policy) gives the same bits as G stacked copies of that set."""
    from merlin import grouped_policy as gp

    G = 32
    models, _ = _tasks(device, 1, seed=77)
    one = {n: p.detach().unsqueeze(0) for n, p in models[0].named_parameters()}
    copies = {n: p.expand(G, *p.shape[1:]).contiguous() for n, p in one.items()}
    codes = _codes(device, G, seed=5)
    a = gp.act_parts(gp.pack(one), codes)
    b = gp.act_parts(gp.pack(copies), codes)
    assert torch.equal(a, b)
