"""GPU: the conv1-from-codes HIP kernels (merlin_conv1_lut_fwd/bwd) against PyTorch's
convolution of the rendered frames: forward within fp32 tolerance, and the gradients
w.r.t. both towers' conv1 weight/bias through the einsum'd tables."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _case(device, n=300, seed=0):
    from test_gpu_obs_gae import pack

    rs = np.random.RandomState(seed)
    c = rs.randint(0, 5, size=(n, 49)).astype(np.uint8)
    c[:, 45] = 4
    return c, torch.from_numpy(pack(c)).to(device)


def test_forward_matches_conv2d(golden, oracle, device):
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    codes49, codes = _case(device)
    torch.manual_seed(1)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    idx = torch.randperm(codes.shape[0], device=device)[:200]
    with torch.no_grad():
        P, b = ac.conv1_tables()
        a1 = nat.conv1_lut_fwd(codes, idx, P.contiguous(), b.contiguous())
        frames = nat.expand_obs(codes, index=idx, scale=1.0 / 255.0)
        for t, tower in enumerate((ac.actor_extractor, ac.critic_extractor)):
            ref = torch.relu(F.conv2d(frames, tower.network[0].weight, tower.network[0].bias, stride=4))
            torch.testing.assert_close(a1[t], ref, rtol=1e-5, atol=1e-5)


def test_backward_matches_conv2d(device):
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    _, codes = _case(device, n=2500, seed=3)
    torch.manual_seed(2)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    idx = torch.randint(0, codes.shape[0], (2000,), device=device)
    g = torch.randn(2, 2000, 32, 13, 13, device=device)
    from merlin.actor_critic import _Conv1FromCodes

    P, b = ac.conv1_tables()
    (_Conv1FromCodes.apply(P, b, codes, idx) * g).sum().backward()
    mine = [(t.network[0].weight.grad.clone(), t.network[0].bias.grad.clone())
            for t in (ac.actor_extractor, ac.critic_extractor)]
    ac.zero_grad()
    frames = nat.expand_obs(codes, index=idx, scale=1.0 / 255.0)
    for t, tower in enumerate((ac.actor_extractor, ac.critic_extractor)):
        (torch.relu(F.conv2d(frames, tower.network[0].weight, tower.network[0].bias, stride=4)) * g[t]).sum().backward()
        for got, ref in zip(mine[t], (tower.network[0].weight.grad, tower.network[0].bias.grad)):
            rel = ((got - ref).norm() / ref.norm()).item()
            assert rel < 1e-5, rel


def test_act_evaluate_codes_match_frames(device):
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    _, codes = _case(device, n=512, seed=4)
    torch.manual_seed(5)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    acts = torch.randint(0, 3, (512,), device=device)
    with torch.no_grad():
        lp1, e1, v1 = ac.evaluate_codes(codes, acts)
        lp2, e2, v2 = ac.evaluate(nat.expand_obs(codes, scale=1.0 / 255.0), acts, prescaled=True)
        a3, lp3, v3 = ac.act_codes(codes, deterministic=True)
        a4, lp4, v4 = ac.act(nat.expand_obs(codes, layout="nhwc"), deterministic=True)
    torch.testing.assert_close(lp1, lp2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1, e2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v1, v2, rtol=1e-5, atol=1e-5)
    assert (a3 == a4).float().mean() > 0.99
    torch.testing.assert_close(v3, v4, rtol=1e-5, atol=1e-5)


def test_ppo_sgd_codes_vs_frames(golden, oracle, device):
    """One update through conv1-from-codes == the frame path on identical inputs."""
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO
    from test_gpu_obs_gae import pack

    g = golden("update_ref")
    B, MB, EPOCHS = (int(x) for x in g["cfg"])
    codes = torch.from_numpy(pack(g["codes"])).to(device)
    perms = torch.from_numpy(g["perms"])
    t = lambda k, dt=torch.float32: torch.from_numpy(g[k]).to(device=device, dtype=dt)  # noqa: E731
    rs = np.random.RandomState(4)
    adv = torch.from_numpy(rs.randn(B).astype(np.float32)).to(device)
    ret = torch.from_numpy(rs.randn(B).astype(np.float32)).to(device)
    res = []
    for lut in (True, False):
        env = MerlinVecEnv(B, "mediumhard", seed=1, device=device)
        torch.manual_seed(0)
        agent = PPO(env, batch_size=B, minibatch_size=MB, update_epochs=EPOCHS, ent_coef=0.05, device=device,
                    perm_fn=lambda n, e: perms[e], conv1_from_codes=lut)
        s = agent._sgd(B, codes, None, t("actions", torch.int64), t("logp"), adv, ret)
        res.append((s, [p.detach().clone() for p in agent.ac.parameters()]))
    (s1, p1), (s2, p2) = res
    for k in s1:
        assert abs(s1[k] - s2[k]) <= 1e-4 * max(1.0, abs(s2[k])), k
    for a, b in zip(p1, p2):
        assert ((a - b).norm() / b.norm()).item() < 1e-5


def _im2col(a, k, s):
    n, C = a.shape[0], a.shape[1]
    u = F.unfold(a, kernel_size=k, stride=s)
    P = u.shape[-1]
    return u.view(n, C, k * k, P).permute(0, 3, 2, 1).reshape(n * P, k * k * C)


def test_tower_glue_kernels_match_torch(device):
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    _, codes = _case(device, n=700, seed=8)
    torch.manual_seed(9)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    idx = torch.randint(0, 700, (333,), device=device)
    with torch.no_grad():
        P, b1 = ac.conv1_tables()
        A2 = nat.conv2_im2col_fwd(codes, idx, P.contiguous(), b1.contiguous())
        frames = nat.expand_obs(codes, index=idx, scale=1.0 / 255.0)
        towers = (ac.actor_extractor.network, ac.critic_extractor.network)
        for t, net in enumerate(towers):
            ref = _im2col(torch.relu(net[0](frames)), 4, 2)
            torch.testing.assert_close(A2[t], ref, rtol=1e-5, atol=1e-5)
        Z2 = torch.randn(2, 333 * 25, 64, device=device)
        b2 = torch.randn(2, 64, device=device)
        A3 = nat.conv3_im2col_fwd(Z2, b2)
        for t in range(2):
            a2 = torch.relu(Z2[t] + b2[t]).view(333, 5, 5, 64).permute(0, 3, 1, 2)
            assert torch.equal(A3[t], _im2col(a2, 3, 1))
    # col2im3 backward == autograd of the torch im2col
    Z2.requires_grad_(True)
    g = torch.randn(2, 333 * 9, 576, device=device)
    ref = torch.autograd.grad(
        torch.stack([_im2col(torch.relu(Z2[t] + b2[t]).view(333, 5, 5, 64).permute(0, 3, 1, 2), 3, 1)
                     for t in range(2)]).mul(g).sum(), Z2)[0]
    mine = nat.conv3_col2im_bwd(g, Z2.detach(), b2)
    torch.testing.assert_close(mine, ref, rtol=1e-5, atol=1e-5)


def test_gemm_tower_forward_and_grads_match_frames(device):
    """CNNActorCritic codes path (GEMM tower) vs the reference-structured frame path:
    outputs and every parameter gradient of a policy/value loss."""
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    _, codes = _case(device, n=1500, seed=10)
    idx = torch.randint(0, 1500, (1024,), device=device)
    acts = torch.randint(0, 3, (1024,), device=device)
    torch.manual_seed(11)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)

    def loss_of(lp, ent, v):
        return -(lp.exp() * 0.7).mean() + 0.5 * (v ** 2).mean() - 0.05 * ent.mean()

    lp1, e1, v1 = ac.evaluate_codes(codes, acts, index=idx)
    loss_of(lp1, e1, v1).backward()
    g1 = [p.grad.clone() for p in ac.parameters()]
    ac.zero_grad()
    frames = nat.expand_obs(codes, index=idx, scale=1.0 / 255.0)
    lp2, e2, v2 = ac.evaluate(frames, acts, prescaled=True)
    loss_of(lp2, e2, v2).backward()
    g2 = [p.grad.clone() for p in ac.parameters()]
    torch.testing.assert_close(lp1, lp2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1, e2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v1, v2, rtol=1e-5, atol=1e-5)
    for (name, _), a, b in zip(ac.named_parameters(), g1, g2):
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        assert rel < 1e-4, (name, rel)
