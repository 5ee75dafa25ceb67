"""GPU: merlin_ppo_loss (csrc/merlin_loss.hip) against the reference's loss formulation
(src/ppo.py:136-150) written in torch with autograd, on minibatches whose samples repeat frames
(the update's distinct-frame evaluation): loss, the five update statistics, and the gradient
with respect to the per-frame logits / values.  Tolerances: fp32 sums in a different order."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_loss(logits, value, inv, actions, lp_old, adv, ret, clip, vf, ent_coef):
    lg, v = logits.index_select(0, inv), value.index_select(0, inv)
    logp_all = lg - lg.logsumexp(-1, keepdim=True)
    probs = torch.softmax(logp_all, -1)
    logp = logp_all.gather(-1, actions.unsqueeze(-1)).squeeze(-1)
    entropy = -(torch.clamp(logp_all, min=torch.finfo(torch.float32).min) * probs).sum(-1)
    ratio = torch.exp(logp - lp_old)
    pi_loss = -torch.min(ratio * adv, torch.clamp(ratio, 1 - clip, 1 + clip) * adv).mean()
    v_loss = ((v - ret) ** 2).mean()
    ent = entropy.mean()
    loss = pi_loss + vf * v_loss - ent_coef * ent
    with torch.no_grad():
        kl = (lp_old - logp).mean()
        cf = (torch.abs(ratio - 1.0) > clip).float().mean()
    return loss, torch.stack([pi_loss, v_loss, ent, kl, cf]).double()


@pytest.mark.parametrize("U,n,A,indexed", [(1, 1, 3, False), (1, 3000, 3, True), (37, 500, 3, True), (5000, 131072 // 8, 3, True),
                                           (300, 4000, 7, False)])
def test_ppo_loss_matches_torch(device, U, n, A, indexed):
    from merlin import _native as nat
    from merlin.ppo import _PPOLoss
    from merlin.windows import MinibatchWindows, _frame_csr

    g = torch.Generator(device=device)
    g.manual_seed(U + n)
    # skewed frame multiplicities; every frame has at least one sample
    inv = torch.cat([torch.arange(U, device=device),
                     (torch.rand(n - U, device=device, generator=g) ** 3 * U).long()])[torch.randperm(n, device=device, generator=g)]
    B = 3 * n if indexed else n
    sample_index = torch.randperm(B, device=device, generator=g)[:n] if indexed else None
    actions = torch.randint(0, A, (B,), device=device, generator=g)
    logits = torch.randn(U, A, device=device, generator=g)
    value = torch.randn(U, device=device, generator=g)
    lp_old = torch.log_softmax(logits.index_select(0, inv) + 0.2 * torch.randn(n, A, device=device, generator=g), -1)
    lp_old = lp_old.gather(-1, actions[sample_index if indexed else slice(None)].unsqueeze(-1)).squeeze(-1)
    lp_full = torch.zeros(B, device=device)
    adv = torch.randn(B, device=device, generator=g)
    ret = torch.randn(B, device=device, generator=g)
    si = sample_index if indexed else torch.arange(n, device=device)
    lp_full[si] = lp_old
    lp_full[si[: n // 10]] = lp_old[: n // 10] + 0.5  # some ratios far outside the clip range
    sk, perm = torch.sort(inv, stable=True)
    new = torch.ones(n, dtype=torch.bool, device=device)
    new[1:] = sk[1:] != sk[:-1]
    mb = MinibatchWindows(None, inv, None, perm.to(torch.int32), _frame_csr(torch.nonzero(new).squeeze(1), n))
    clip, vf, ent_coef = 0.2, 0.5, 0.05

    lr = logits.clone().requires_grad_(True)
    vr = value.clone().requires_grad_(True)
    ref_loss, ref_stats = _torch_loss(lr, vr, inv, actions[si], lp_full[si], adv[si], ret[si], clip, vf, ent_coef)
    ref_loss.backward()

    # the kernel adds the heads' biases itself: pass the logits / value without them
    ba = torch.randn(A, device=device, generator=g).requires_grad_(True)
    bc = torch.randn(1, device=device, generator=g).requires_grad_(True)
    lm = (logits - ba.detach()).requires_grad_(True)
    vm = (value - bc.detach()).requires_grad_(True)
    stats = torch.zeros(6, dtype=torch.float64, device=device)
    loss = _PPOLoss.apply(lm, vm, ba, bc, mb, sample_index, actions, lp_full, adv, ret, clip, vf, ent_coef, stats)
    (2.0 * loss).backward()
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(stats[:5], ref_stats, rtol=1e-5, atol=1e-6)
    assert stats[5] == 0
    torch.testing.assert_close(lm.grad, 2.0 * lr.grad, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(vm.grad, 2.0 * vr.grad, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(ba.grad, 2.0 * lr.grad.sum(0), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(bc.grad, 2.0 * vr.grad.sum(0, keepdim=True), rtol=1e-4, atol=1e-6)
    # fixed order: a second call gives the same bits
    l2, d2, v2, _, _ = nat.ppo_loss(logits, value, mb.offs, mb.order, inv, sample_index, actions, lp_full, adv, ret, clip, vf,
                              ent_coef)
    l1, d1, v1, _, _ = nat.ppo_loss(logits, value, mb.offs, mb.order, inv, sample_index, actions, lp_full, adv, ret, clip, vf,
                              ent_coef)
    assert torch.equal(l1, l2) and torch.equal(d1, d2) and torch.equal(v1, v2)
    # merlin_ppo_loss_absmax: the same outputs, and the per-output maxima of |dlogits| / |dvalue| (the bound the
    # heads' backward scales dz's planes by) exactly
    gm = torch.zeros(9, dtype=torch.int32, device=device)
    l3, d3, v3, _, _ = nat.ppo_loss(logits, value, mb.offs, mb.order, inv, sample_index, actions, lp_full, adv, ret,
                                    clip, vf, ent_coef, grad_absmax=gm)
    assert torch.equal(l3, l1) and torch.equal(d3, d1) and torch.equal(v3, v1)
    want = torch.zeros(9, dtype=torch.float32, device=device)
    want[:A] = d1.abs().amax(0)
    want[8] = v1.abs().amax()
    assert torch.equal(gm.view(torch.float32), want)


def test_ppo_loss_bad_action_is_nan(device):
    from merlin import _native as nat

    logits, value = torch.zeros(2, 3, device=device), torch.zeros(2, device=device)
    offs = torch.tensor([0, 1, 2], dtype=torch.int32, device=device)
    order = torch.tensor([0, 1], dtype=torch.int32, device=device)
    actions = torch.tensor([1, 5], device=device)
    z = torch.zeros(2, device=device)
    loss = nat.ppo_loss(logits, value, offs, order, torch.arange(2, device=device), None, actions, z, z + 1, z, 0.2, 0.5, 0.05)[0]
    assert torch.isnan(loss)
