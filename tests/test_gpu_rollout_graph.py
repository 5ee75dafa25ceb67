"""GPU: the acting path with per-rollout weight layouts (CNNActorCritic.act_codes_packed) ==
act_codes, and the captured rollout (PPO._capture_rollout: one HIP graph per rollout) == eager
launches: its observations, rewards and dones replay bit-exact through an eager env fed its
actions, its log-probs / values re-evaluate to the stored ones with the weights of that
rollout, and every replay draws fresh actions."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _observable_codes(device, n, seed):
    """Frames an env can show: random tile classes 0..3 (empty-dark, empty-lit, wall, goal) with the agent's tile
    (class 4) at its view cell (3, 6) only -- the acting table's compact keys cover exactly these (merlin/windows.py
    compact_window_keys) -- followed by real observations of a stepped vector env."""
    import numpy as np

    from merlin import MerlinVecEnv
    from test_gpu_obs_gae import pack

    rs = np.random.RandomState(seed)
    c = rs.randint(0, 4, size=(n, 49)).astype(np.uint8)
    c[:, 45] = 4
    rand = torch.from_numpy(pack(c)).to(device)
    env = MerlinVecEnv(n, "mediumhard", seed=seed, device=device)
    frames = [env.reset().clone()]
    g = torch.Generator(device=device).manual_seed(seed)
    for _ in range(3):
        frames.append(env.step(torch.randint(0, 3, (n,), device=device, generator=g))[0].clone())
    env.close()
    return torch.cat([rand] + frames)


@pytest.mark.parametrize("frames", [None, 1000])
def test_packed_act_matches_act_codes(device, frames):
    """Both acting layouts of rollout_pack: the all-windows table (large rollouts) and the per-frame
    conv2 lookups + conv3 GEMM (small rollouts, no 2-GB table)."""
    from merlin.actor_critic import CNNActorCritic

    codes = _observable_codes(device, 700, seed=3)
    torch.manual_seed(4)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    with torch.no_grad():
        a1, lp1, v1 = ac.act_codes(codes, deterministic=True)
        pack = ac.rollout_pack(frames=frames)
        assert ("Qall" in pack) == (frames is None)
        a2, lp2, v2 = ac.act_codes_packed(codes, pack, deterministic=True)
    same = a1 == a2
    assert same.float().mean() > 0.99
    torch.testing.assert_close(lp1[same], lp2[same], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v1, v2, rtol=1e-5, atol=1e-5)


def test_codes_conv3_matches_im2col_path(device):
    """merlin_tower_codes_conv3 over the all-windows table of rollout_pack() == conv2 lookups ->
    conv3 im2col -> GEMM -> bias + ReLU (the per-frame path of evaluate_codes) on the same frames."""
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    codes = _observable_codes(device, 900, seed=5)
    torch.manual_seed(6)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    with torch.no_grad():
        pack = ac.rollout_pack()
        assert pack["Qall"].shape == (2, nat.ALL_WINDOWS, 576)
        Y3 = nat.codes_conv3(codes, pack["Qall"], pack["b3"])
        A3 = nat.conv3_im2col_fwd(nat.conv2_lut_fwd(codes, None, ac.conv2_tables().contiguous()),
                                  torch.stack([ea[2].bias, ec[2].bias]).contiguous())
        W3t = torch.stack([ea[4].weight, ec[4].weight]).permute(0, 3, 4, 2, 1).reshape(2, 576, 64)
        ref = torch.relu(torch.bmm(A3, W3t) + torch.stack([ea[4].bias, ec[4].bias]).unsqueeze(1))
    torch.testing.assert_close(Y3, ref, rtol=1e-5, atol=1e-5)


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



def test_codes_conv3_flags_frames_that_are_no_observation(device):
    """The compact acting table holds windows of classes 0..3 plus the agent tile at view cell (3, 6) only
    (csrc/merlin_window.hip k_codes_conv3).  A frame outside that set -- the agent tile elsewhere, or missing at
    (3, 6) -- raises MERLIN_DEVERR_BAD_TILE (merlin_tower_errors) instead of being read silently as another window;
    observations leave the flags clear."""
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(6)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    with torch.no_grad():
        pack = ac.rollout_pack()
    nat.tower_errors(device, raise_on_error=False)  # clear
    codes = _observable_codes(device, 300, seed=9)
    nat.codes_conv3(codes, pack["Qall"], pack["b3"])
    assert nat.tower_errors(device, raise_on_error=False) == 0
    import numpy as np

    from test_gpu_obs_gae import pack as pack_codes

    c = np.random.RandomState(9).randint(0, 4, size=(64, 49)).astype(np.uint8)
    c[:, 45] = 4
    for cell, cls in ((10, 4), (45, 2)):  # an agent tile at (3, 1); no agent tile at (3, 6)
        b = c.copy()
        b[7, cell] = cls
        bad = torch.from_numpy(pack_codes(b)).to(device)
        nat.codes_conv3(bad, pack["Qall"], pack["b3"])
        assert nat.tower_errors(device, raise_on_error=False) == nat.DEVERR_BAD_TILE, cell
        nat.codes_conv3(bad, pack["Qall"], pack["b3"])
        with pytest.raises(nat.MerlinNativeError):
            nat.tower_errors(device)
    assert nat.tower_errors(device, raise_on_error=False) == 0
