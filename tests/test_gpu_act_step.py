"""GPU: the rollout's draw fused into the env step (merlin_env_act_step, round 5) against the two launches it replaces
(merlin_act_draw, then merlin_env_step): the same actions / log-probs / values and the same env trajectory bit for
bit, over many steps with frequent episode ends (short max_steps, so resets take look-ahead slots and, when a slot is
empty, take the k_env_fallback path), sampled and deterministic, 16x16 and the 22x22 layout."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("difficulty,size,det", [("mediumhard", 16, False), ("mediumhard", 16, True),
                                                 ("hard", 22, False)])
def test_act_step_matches_draw_then_step(device, difficulty, size, det):
    from merlin import MerlinVecEnv
    from merlin import _native as nat

    N, T, P = 777, 40, 4
    envs = [MerlinVecEnv(N, difficulty, size=size, seed=31, device=device, max_steps=9, env_offset=5)
            for _ in range(2)]
    for e in envs:
        e.set_refill_interval(0)  # no refills at all: every second reset finds its slot empty
        e.reset()
    g = torch.Generator(device=device).manual_seed(size + det)
    ba = torch.randn(3, device=device, generator=g)
    bc = torch.randn(1, device=device, generator=g)
    epoch = torch.tensor([3], dtype=torch.int64, device=device)
    bufs = [{k: torch.empty(N, dtype=dt, device=device) for k, dt in
             (("a", torch.int64), ("lp", torch.float32), ("v", torch.float32), ("r", torch.float32),
              ("d", torch.float32), ("er", torch.float64), ("el", torch.int32))} for _ in range(2)]
    obs = [torch.empty(N, 8, dtype=torch.int32, device=device) for _ in range(2)]
    ended = 0
    for t in range(T):
        part = torch.randn(2, P, N, 4, device=device, generator=g)
        b0, b1 = bufs
        nat.act_draw(part, ba, bc, det, seed=11, epoch=epoch, step=t, out=(b0["a"], b0["lp"], b0["v"]), env_offset=5)
        envs[0].step_into(b0["a"], obs[0], b0["r"], None, None, b0["d"], b0["er"], b0["el"])
        envs[1].act_step_into(part, ba, bc, (b1["a"], b1["lp"], b1["v"]), obs[1], b1["r"], None, None, b1["d"],
                              b1["er"], b1["el"], deterministic=det, seed=11, epoch=epoch, step=t)
        torch.cuda.synchronize()
        for k in b0:
            d = b0["d"] > 0
            if k in ("er", "el"):  # written only where an episode ended
                assert torch.equal(b0[k][d], b1[k][d]), (t, k)
            else:
                assert torch.equal(b0[k], b1[k]), (t, k)
        assert torch.equal(obs[0], obs[1]), t
        ended += int((b0["d"] > 0).sum())
    s0, s1 = envs[0].get_state(), envs[1].get_state()
    for k in s0:
        assert (s0[k] == s1[k]).all(), k
    assert ended > 2 * N  # most envs went through several episodes (resets from slots and generated in-launch)
    for e in envs:
        e.errors()
        e.close()
