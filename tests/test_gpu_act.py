"""GPU: merlin_act_heads (csrc/merlin_act.hip), the acting tail of CNNActorCritic.act
(src/actor_critic.py:48-55), against the same math in torch fp32: relu(z + b4) -> actor /
critic heads -> log_softmax -> argmax (deterministic) or a Categorical draw.  Tolerances: fp32
dot products summed in a different order (1e-4 relative).  The stochastic draw is checked by
its law (empirical action frequencies vs softmax, chi-square bound), its logp (= log_softmax
at the drawn action), its determinism for a fixed (seed, epoch, step) and its freshness when
the epoch counter moves (what the rollout graph replays rely on)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_heads(z, b4, wa, ba, wc, bc):
    h = torch.relu(z + b4[:, None, :])
    logits = h[0] @ wa.T + ba
    value = h[1] @ wc.reshape(-1) + bc.reshape(())
    return logits.log_softmax(-1), value


def _inputs(device, n, H, A, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    r = lambda *s: torch.randn(*s, device=device, generator=g)  # noqa: E731
    return r(2, n, H), r(2, H) * 0.1, r(A, H) * 0.05, r(A) * 0.1, r(1, H) * 0.05, r(1) * 0.1


@pytest.mark.parametrize("n,H,A", [(1, 4, 1), (3, 64, 3), (4097, 512, 3), (1000, 260, 7), (77, 512, 8)])
def test_act_heads_deterministic_matches_torch(device, n, H, A):
    from merlin import _native as nat

    z, b4, wa, ba, wc, bc = _inputs(device, n, H, A, n + H + A)
    action, logp, value = nat.act_heads(z, b4, wa, ba, wc, bc, deterministic=True)
    torch.cuda.synchronize()
    lp_all, v_ref = _torch_heads(z, b4, wa, ba, wc, bc)
    torch.testing.assert_close(value, v_ref, rtol=1e-4, atol=1e-4)
    # argmax may differ from torch's only where two logits tie within fp32 summation noise
    a_ref = lp_all.argmax(-1)
    top2 = lp_all.topk(min(2, A), -1).values
    near_tie = (top2[:, 0] - top2[:, -1] < 1e-4) if A > 1 else torch.zeros(n, dtype=torch.bool, device=device)
    assert bool(((action == a_ref) | near_tie).all())
    torch.testing.assert_close(logp, lp_all.gather(-1, action[:, None]).squeeze(-1), rtol=1e-4, atol=1e-4)


def test_act_heads_sample_law_and_replay(device):
    from merlin import _native as nat

    n, H, A = 65536, 512, 3
    z, b4, wa, ba, wc, bc = _inputs(device, n, H, A, 7)
    # one shared row for every env so the empirical frequencies estimate one distribution
    z = z[:, :1].expand(2, n, H).contiguous()
    epoch = torch.zeros(1, dtype=torch.int64, device=device)
    a1, lp1, _ = nat.act_heads(z, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=5)
    a1, lp1 = a1.clone(), lp1.clone()
    a2, _, _ = nat.act_heads(z, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=5)
    assert torch.equal(a1, a2)  # counter-based: same key, same draw
    lp_all, _ = _torch_heads(z[:, :1], b4, wa, ba, wc, bc)
    p = lp_all[0].exp().double()
    torch.testing.assert_close(lp1, lp_all[0][a1], rtol=1e-4, atol=1e-4)
    counts = torch.bincount(a1, minlength=A).double()
    chi2 = float((((counts - n * p) ** 2) / (n * p).clamp_min(1e-12)).sum())
    assert chi2 < 30.0, (counts.tolist(), (n * p).tolist())  # df = 2: p-value ~3e-7
    epoch.add_(1)
    a3, _, _ = nat.act_heads(z, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=5)
    a4, _, _ = nat.act_heads(z, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=6)
    assert not torch.equal(a1, a3) and not torch.equal(a3, a4)


def test_act_heads_writes_into_storage(device):
    from merlin import _native as nat

    n, H, A = 300, 64, 3
    z, b4, wa, ba, wc, bc = _inputs(device, n, H, A, 11)
    act = torch.full((2, n), -1, dtype=torch.int64, device=device)
    lp = torch.full((2, n), 9.0, device=device)
    val = torch.full((2, n), 9.0, device=device)
    nat.act_heads(z, b4, wa, ba, wc, bc, deterministic=True, out=(act[1], lp[1], val[1]))
    torch.cuda.synchronize()
    assert bool((act[0] == -1).all()) and bool((lp[0] == 9.0).all()) and bool((val[0] == 9.0).all())
    assert bool(((act[1] >= 0) & (act[1] < A)).all()) and bool((lp[1] <= 0).all())
