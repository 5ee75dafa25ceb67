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


def test_act_heads_non_finite_logits_give_sentinel_and_env_rejects_it(device):
    """A diverged policy (NaN / inf logits) must not silently act: the reference's
    Categorical(logits) raises; merlin_act_heads writes action -1 and the next env step raises
    MERLIN_DEVERR_BAD_ACTION through MerlinVecEnv.errors()."""
    from merlin import MerlinVecEnv
    from merlin import _native as nat

    n, H, A = 64, 64, 3
    z, b4, wa, ba, wc, bc = _inputs(device, n, H, A, 13)
    z[0, 5, 3] = float("nan")
    z[0, 9, :] = float("inf")
    epoch = torch.zeros(1, dtype=torch.int64, device=device)
    for det in (True, False):
        action, _, _ = nat.act_heads(z, b4, wa, ba, wc, bc, deterministic=det, seed=1, epoch=epoch)
        assert int(action[5]) == -1 and int(action[9]) == -1
        ok = torch.ones(n, dtype=torch.bool, device=device)
        ok[5] = ok[9] = False
        assert bool(((action[ok] >= 0) & (action[ok] < A)).all())
    env = MerlinVecEnv(n, "mediumhard", seed=3, device=device)
    env.reset()
    env.step(action)
    with pytest.raises(nat.MerlinNativeError, match="non-finite"):
        env.errors()


def test_act_heads_keys_on_the_global_env_index(device):
    """data-parallel ranks (same torch seed on every rank, ppo_train.py set_seed) must not
    share sampling noise.  The draw is keyed by env_offset + env: rank r (env_offset r*n) draws
    differently from rank 0 for identical logits, and exactly what one process over the 2n
    concatenated envs draws for those envs."""
    from merlin import _native as nat

    n, H, A = 4096, 64, 3
    z, b4, wa, ba, wc, bc = _inputs(device, n, H, A, 17)
    z = z[:, :1].expand(2, n, H).contiguous()  # identical logits for every env
    epoch = torch.full((1,), 3, dtype=torch.int64, device=device)
    r0, _, _ = nat.act_heads(z, b4, wa, ba, wc, bc, seed=9, epoch=epoch, step=2, env_offset=0)
    r1, _, _ = nat.act_heads(z, b4, wa, ba, wc, bc, seed=9, epoch=epoch, step=2, env_offset=n)
    assert (r0 != r1).float().mean() > 0.2
    zz = torch.cat([z, z], 1)
    both, _, _ = nat.act_heads(zz, b4, wa, ba, wc, bc, seed=9, epoch=epoch, step=2)
    assert torch.equal(both[:n], r0) and torch.equal(both[n:], r1)


@pytest.mark.parametrize("n,A", [(4096, 3), (1000, 4), (77, 1)])
def test_act_draw_from_gemm_heads_matches_act_heads(device, n, A):
    """The acting path's heads folded into fc1's h3 GEMM (merlin_h3_gemm_nt_heads without h, then merlin_act_draw)
    == fc1's GEMM then merlin_act_heads: deterministic actions equal (no near-ties at these scales), logp / value
    within fp32 reordering, and a sampled draw keyed by the same (seed, epoch, step, env) picks the same actions."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(n + A)
    a3 = torch.relu(torch.randn(2, n, 576, device=device, generator=g))
    W4 = torch.randn(2, 512, 576, device=device, generator=g) / 24
    b4 = torch.randn(2, 512, device=device, generator=g) * 0.1
    wa = torch.randn(A, 512, device=device, generator=g) * 0.05
    ba = torch.randn(A, device=device, generator=g) * 0.1
    wc = torch.randn(1, 512, device=device, generator=g) * 0.05
    bc = torch.randn(1, device=device, generator=g) * 0.1
    am3, amW = nat.h3_amax(a3), nat.h3_amax(W4)
    P4 = nat.h3_split(W4, amW)
    cfg = nat.H3_NT_CFG["rollout"]
    z = nat.h3_gemm_nt(a3, am3, P4, amW, cfg=cfg)
    part = nat.h3_gemm_nt_heads(a3, am3, P4, amW, b4, wa, wc, cfg=cfg, partials_only=True)
    epoch = torch.tensor([3], dtype=torch.int64, device=device)
    for det in (True, False):
        a1, lp1, v1 = nat.act_heads(z, b4, wa, ba, wc, bc, deterministic=det, seed=5, epoch=epoch, step=2)
        a2, lp2, v2 = nat.act_draw(part, ba, bc, deterministic=det, seed=5, epoch=epoch, step=2)
        assert float((a1 == a2).float().mean()) >= 0.999
        same = a1 == a2
        torch.testing.assert_close(lp2[same], lp1[same], rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(v2, v1, rtol=1e-4, atol=1e-5)
