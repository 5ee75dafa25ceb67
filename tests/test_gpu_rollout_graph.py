"""GPU: the acting path with per-rollout weight layouts (CNNActorCritic.act_codes_packed) ==
act_codes, and the captured rollout (PPO._capture_rollout: one HIP graph per rollout) == eager
launches: its observations, rewards and dones replay bit-exact through an eager env fed its
actions, its log-probs / values re-evaluate to the stored ones with the weights of that
rollout, and every replay draws fresh actions."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_packed_act_matches_act_codes(device):
    from merlin.actor_critic import CNNActorCritic
    from test_gpu_conv2lut import _codes

    _, codes = _codes(device, 700, seed=3)
    torch.manual_seed(4)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    with torch.no_grad():
        a1, lp1, v1 = ac.act_codes(codes, deterministic=True)
        a2, lp2, v2 = ac.act_codes_packed(codes, ac.rollout_pack(), deterministic=True)
    same = a1 == a2
    assert same.float().mean() > 0.99
    torch.testing.assert_close(lp1[same], lp2[same], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v1, v2, rtol=1e-5, atol=1e-5)


def test_graph_rollout_matches_eager_env(device):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    N, T = 256, 16
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=device, max_steps=12)
    mirror = MerlinVecEnv(N, "mediumhard", seed=777, device=device, max_steps=12)
    torch.manual_seed(0)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=1, ent_coef=0.05, device=device)
    buf = agent.buf
    seen = []
    for it in range(3):
        lv = agent.collect_rollouts()
        assert agent._graph is not None  # captured after the first (eager) rollout
        codes = torch.zeros_like(buf.codes)
        rew, done = torch.zeros_like(buf.rewards), torch.zeros_like(buf.dones)
        mirror.reset(out=codes[0])
        for t in range(T):
            mirror.step_into(buf.actions[t].contiguous(), codes[t + 1], rew[t], None, None, done[t])
        assert torch.equal(codes, buf.codes)
        assert torch.equal(rew, buf.rewards) and torch.equal(done, buf.dones)
        assert (done.sum(0) >= 1).all()  # max_steps 12 < T: every env auto-reset inside the graph
        with torch.no_grad():
            for t in (0, T // 2, T - 1):
                lp, _, v = agent.ac.evaluate_codes(buf.codes[t], buf.actions[t])
                torch.testing.assert_close(lp, buf.logprobs[t], rtol=1e-5, atol=1e-5)
                torch.testing.assert_close(v, buf.values[t], rtol=1e-5, atol=1e-5)
            _, _, v = agent.ac.act_codes(buf.codes[T])
            torch.testing.assert_close(v, buf.last_value, rtol=1e-5, atol=1e-5)
        seen.append(buf.actions.clone())
        agent.update(lv)  # new weights: the next replay must read them in place
    assert not torch.equal(seen[1], seen[2])
    mirror.errors()


def test_act_heads_matches_torch_and_samples_the_policy(device):
    """merlin_act_heads: relu(z + b4) -> heads -> log_softmax == torch; deterministic = argmax;
    the draws follow softmax(logits) (per-env empirical frequencies over many keys) and change
    with the epoch counter."""
    from merlin import _native as nat

    g = torch.Generator(device=device)
    g.manual_seed(5)
    n, H, A = 3000, 512, 3
    z = torch.randn(2, n, H, device=device, generator=g)
    b4 = torch.randn(2, H, device=device, generator=g) * 0.1
    wa = torch.randn(A, H, device=device, generator=g) * 0.05
    ba = torch.randn(A, device=device, generator=g)
    wc = torch.randn(1, H, device=device, generator=g) * 0.05
    bc = torch.randn(1, device=device, generator=g)
    h = torch.relu(z + b4[:, None])
    logits = h[0] @ wa.t() + ba
    logp_all = torch.log_softmax(logits, -1)
    value = (h[1] @ wc.t()).squeeze(-1) + bc
    a, lp, v = nat.act_heads(z, b4, wa, ba, wc, bc, deterministic=True)
    assert torch.equal(a, logits.argmax(-1))
    torch.testing.assert_close(lp, logp_all.gather(-1, a[:, None]).squeeze(-1), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v, value, rtol=1e-5, atol=1e-5)
    # sampling: same frame for every env -> frequencies over 3000 envs x 20 steps ~ softmax
    zz = z[:, :1].expand(2, n, H).contiguous()
    p = torch.softmax(h[0, :1] @ wa.t() + ba, -1)[0]
    epoch = torch.zeros(1, dtype=torch.int64, device=device)
    counts = torch.zeros(A, device=device)
    first = None
    for step in range(20):
        a, lp, _ = nat.act_heads(zz, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=step)
        counts += torch.bincount(a, minlength=A).float()
        torch.testing.assert_close(lp, torch.log(p)[a], rtol=1e-5, atol=1e-5)
        if first is None:
            first = a.clone()
    freq = counts / counts.sum()
    assert (freq - p).abs().max() < 0.01, (freq, p)  # 60k draws: sd < 0.002
    a0, _, _ = nat.act_heads(zz, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=0)
    assert torch.equal(a0, first)  # same key, same draw
    epoch += 1
    a1, _, _ = nat.act_heads(zz, b4, wa, ba, wc, bc, seed=123, epoch=epoch, step=0)
    assert not torch.equal(a1, first)
