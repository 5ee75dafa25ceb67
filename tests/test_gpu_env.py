"""GPU parity: the HIP env kernels (through the C ABI) vs the golden traces and the
C oracle, bit-exact on grid state, agent state, observation codes, reward (f32)
and done flags."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def unpack(codes_i32: torch.Tensor) -> np.ndarray:
    """int32[..., 8] nibble words -> uint8[..., 49] tile classes."""
    w = codes_i32.cpu().numpy().astype(np.uint32).view(np.uint32)
    nib = (w[..., :, None] >> (4 * np.arange(8, dtype=np.uint32))) & 0xF
    return nib.reshape(*w.shape[:-1], 64)[..., :49].astype(np.uint8)


def make_env(n, diff, size, seed, device, **kw):
    from merlin import MerlinVecEnv

    return MerlinVecEnv(n, difficulty=diff, size=size, seed=seed, device=device, **kw)


MAP_KEYS = ["mediumhard_16", "hard_16", "hard_22", "easy_16", "medium_16", "hardest_16"]


@pytest.mark.parametrize("key", MAP_KEYS)
def test_seeded_maps_match_golden(golden, device, key):
    """reset(seed=s) map generation incl. multi-attempt seeds, every generator."""
    g = golden("env_maps")
    diff, size = key.rsplit("_", 1)
    size = int(size)
    seeds = g[key + "_seeds"].astype(np.uint64)
    env = make_env(len(seeds), diff, size, 0, device)
    # per-env explicit seeds: seed(base) gives env i base+i; emulate arbitrary seeds via env_offset=0 & a loop
    import ctypes as C

    from merlin import _native as nat

    nat.check(env._lib.merlin_env_seed(env._h, seeds.ctypes.data_as(C.POINTER(C.c_uint64)), len(seeds),
                                       env._stream))
    env._seeded_once = True
    env.reset()
    st = env.get_state()
    assert (st["cells"] == g[key + "_cells"]).all()
    meta = g[key + "_meta"]
    assert (st["agent_pos"] == meta[:, 0:2]).all()
    assert (st["agent_dir"] == meta[:, 2]).all()
    assert (st["goal_pos"] == meta[:, 3:5]).all()
    assert (st["step_count"] == 0).all()
    flags, _ = env.errors()
    assert flags == 0


@pytest.mark.parametrize("key", ["mediumhard_16", "hard_22", "easy_16"])
def test_rollout_trace_matches_golden(golden, device, key):
    """Seeded reset, then the recorded actions with unseeded auto-reset, one step per launch."""
    g = golden("env_trace")
    diff, size = key.rsplit("_", 1)
    n, T, max_steps, base = (int(x) for x in g[key + "_cfg"])
    env = make_env(n, diff, int(size), base, device, max_steps=max_steps or None)
    obs0 = env.reset().clone()
    assert (unpack(obs0) == g[key + "_codes"][0]).all()
    acts = torch.from_numpy(g[key + "_actions"]).to(device)
    codes = torch.zeros((T, n, 8), dtype=torch.int32, device=device)
    rew = torch.zeros((T, n), dtype=torch.float32, device=device)
    term = torch.zeros((T, n), dtype=torch.uint8, device=device)
    trunc = torch.zeros((T, n), dtype=torch.uint8, device=device)
    done = torch.zeros((T, n), dtype=torch.float32, device=device)
    for t in range(T):
        env.step_into(acts[t].contiguous(), codes[t], rew[t], term[t], trunc[t], done[t])
    assert (unpack(codes) == g[key + "_codes"][1:]).all()
    assert (rew.cpu().numpy() == g[key + "_reward"]).all()
    assert (term.cpu().numpy() == g[key + "_term"]).all()
    assert (trunc.cpu().numpy() == g[key + "_trunc"]).all()
    assert (done.cpu().numpy() == np.maximum(g[key + "_term"], g[key + "_trunc"])).all()
    st = env.get_state()
    ag = g[key + "_agent"][-1]
    assert (st["agent_pos"] == ag[:, 0:2]).all() and (st["agent_dir"] == ag[:, 2]).all()
    assert (st["step_count"] == ag[:, 3]).all()


def test_multistep_launch_equals_single_steps(golden, device):
    """n_steps > 1 in one launch (state kept on chip) == n_steps single launches."""
    g = golden("env_trace")
    key = "mediumhard_16"
    n, T, max_steps, base = (int(x) for x in g[key + "_cfg"])
    env = make_env(n, "mediumhard", 16, base, device, max_steps=max_steps)
    env.reset()
    acts = torch.from_numpy(g[key + "_actions"]).to(device).contiguous()
    codes = torch.zeros((T, n, 8), dtype=torch.int32, device=device)
    rew = torch.zeros((T, n), dtype=torch.float32, device=device)
    done = torch.zeros((T, n), dtype=torch.float32, device=device)
    env.step_into(acts, codes, rew, None, None, done, n_steps=T, action_stride=n)
    assert (unpack(codes) == g[key + "_codes"][1:]).all()
    assert (rew.cpu().numpy() == g[key + "_reward"]).all()


@pytest.mark.parametrize("diff,size", [("mediumhard", 16), ("hard", 22), ("hardest", 16), ("medium", 16)])
def test_large_batch_vs_oracle(oracle, device, diff, size):
    """4096 envs (the BASELINE config width), random actions incl. a forward bias so goals
    are reached, short max_steps to exercise truncation + auto-reset; every env checked
    against the C oracle."""
    n, T, max_steps = 4096, 96, 40
    rs = np.random.RandomState(size)
    acts = rs.choice([0, 1, 2], size=(T, n), p=[0.15, 0.15, 0.7]).astype(np.int64)
    env = make_env(n, diff, size, 777, device, max_steps=max_steps)
    obs0 = env.reset().clone()
    codes = torch.zeros((T, n, 8), dtype=torch.int32, device=device)
    rew = torch.zeros((T, n), dtype=torch.float32, device=device)
    term = torch.zeros((T, n), dtype=torch.uint8, device=device)
    trunc = torch.zeros((T, n), dtype=torch.uint8, device=device)
    ta = torch.from_numpy(acts).to(device)
    for t in range(T):
        env.step_into(ta[t].contiguous(), codes[t], rew[t], term[t], trunc[t])
    seeds = np.arange(777, 777 + n, dtype=np.uint64)
    ocodes, orew, oterm, otrunc, oagent = oracle.batch_rollout(seeds, acts, size=size, difficulty=diff,
                                                               max_steps=max_steps)
    assert (unpack(obs0) == ocodes[0]).all()
    assert (unpack(codes) == ocodes[1:]).all()
    assert (rew.cpu().numpy() == orew).all()
    assert (term.cpu().numpy() == oterm).all() and (trunc.cpu().numpy() == otrunc).all()
    assert oterm.sum() > 0 and otrunc.sum() > 0
    st = env.get_state()
    assert (st["agent_pos"] == oagent[-1][:, 0:2]).all() and (st["agent_dir"] == oagent[-1][:, 2]).all()


@pytest.mark.parametrize("mode", ["never", "side_stream_every_step", "every_step", "multistep"])
def test_lookahead_refill_modes_vs_oracle(oracle, device, mode):
    """The look-ahead map slots (merlin_env_set_refill_interval / merlin_env_refill) never change
    results: with no refills at all (every later reset generates in k_env_fallback), a refill on a
    side stream after every step (PPO's rollout), the library's own refill after every step, and
    n_steps > 1 launches (resets generate in the step kernel) -- all equal the C oracle.  Short
    episodes (max_steps 6, forward-biased actions) so envs reset several times per refill window."""
    n, T, max_steps = 2048, 64, 6
    rs = np.random.RandomState(5)
    acts = rs.choice([0, 1, 2], size=(T, n), p=[0.1, 0.1, 0.8]).astype(np.int64)
    env = make_env(n, "mediumhard", 16, 4242, device, max_steps=max_steps)
    env.set_refill_interval({"never": 0, "side_stream_every_step": 0, "every_step": 1, "multistep": 16}[mode])
    env.reset()
    codes = torch.zeros((T, n, 8), dtype=torch.int32, device=device)
    rew = torch.zeros((T, n), dtype=torch.float32, device=device)
    done = torch.zeros((T, n), dtype=torch.float32, device=device)
    ta = torch.from_numpy(acts).to(device)
    if mode == "multistep":
        env.step_into(ta, codes, rew, None, None, done, n_steps=T, action_stride=n)
    else:
        main, side = torch.cuda.current_stream(device), torch.cuda.Stream(device)
        for t in range(T):
            if mode == "side_stream_every_step" and t > 0:
                main.wait_stream(side)
            env.step_into(ta[t].contiguous(), codes[t], rew[t], None, None, done[t])
            if mode == "side_stream_every_step":
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    env.refill()
        main.wait_stream(side)
    torch.cuda.synchronize(device)
    ocodes, orew, oterm, otrunc, _ = oracle.batch_rollout(np.arange(4242, 4242 + n, dtype=np.uint64), acts,
                                                          size=16, difficulty="mediumhard", max_steps=max_steps)
    assert (unpack(codes) == ocodes[1:]).all()
    assert (rew.cpu().numpy() == orew).all()
    assert (done.cpu().numpy() == np.maximum(oterm, otrunc)).all()
    # several resets of one env inside 16 steps (the slot is already used): the fallback path ran
    per_env = np.maximum(oterm, otrunc)[:16].sum(0)
    assert (per_env >= 2).sum() > n // 2
    flags, _ = env.errors()
    assert flags == 0


@pytest.mark.parametrize("stuck,explore", [(True, False), (False, True), (True, True)])
def test_wrapper_flags_vs_oracle(oracle, device, stuck, explore):
    n, T = 512, 120
    rs = np.random.RandomState(1)
    acts = rs.choice([0, 1, 2], size=(T, n), p=[0.3, 0.3, 0.4]).astype(np.int64)
    env = make_env(n, "mediumhard", 16, 31, device, max_steps=50, stuck_penalty=stuck,
                   exploration_bonus=explore, bonus=0.05)
    env.reset()
    rew = torch.zeros((T, n), dtype=torch.float32, device=device)
    ta = torch.from_numpy(acts).to(device)
    for t in range(T):
        env.step_into(ta[t].contiguous(), None, rew[t])
    _, orew, _, _, _ = oracle.batch_rollout(np.arange(31, 31 + n, dtype=np.uint64), acts, max_steps=50,
                                            stuck=stuck, explore=explore, explore_bonus=0.05)
    assert (rew.cpu().numpy() == orew).all()
    assert (orew < 0).any() == stuck


def test_episode_stats(device):
    n, T = 256, 200
    env = make_env(n, "mediumhard", 16, 5, device, max_steps=30)
    env.reset()
    acts = torch.randint(0, 3, (T, n), device=device)
    rew = torch.zeros((T, n), dtype=torch.float32, device=device)
    done = torch.zeros((T, n), dtype=torch.float32, device=device)
    epr = torch.zeros((T, n), dtype=torch.float64, device=device)
    epl = torch.zeros((T, n), dtype=torch.int32, device=device)
    for t in range(T):
        env.step_into(acts[t].contiguous(), None, rew[t], None, None, done[t], epr[t], epl[t])
    r, d, R, L = rew.cpu().numpy(), done.cpu().numpy(), epr.cpu().numpy(), epl.cpu().numpy()
    for i in range(0, n, 17):
        acc, ln = 0.0, 0
        for t in range(T):
            acc += float(r[t, i])
            ln += 1
            if d[t, i]:
                assert L[t, i] == ln and abs(R[t, i] - acc) < 1e-6
                acc, ln = 0.0, 0


def test_bad_action_flag(device):
    from merlin import _native as nat

    env = make_env(64, "mediumhard", 16, 1, device)
    env.reset()
    a = torch.full((64,), 2, dtype=torch.int64, device=device)
    a[7] = 5
    env.step_into(a)
    with pytest.raises(nat.MerlinNativeError):
        env.errors()
    assert env.errors()[0] == 0  # read-and-clear


def test_reset_is_deterministic_and_continues_stream(device):
    e1 = make_env(128, "mediumhard", 16, 42, device)
    e2 = make_env(128, "mediumhard", 16, 42, device)
    a = e1.reset().clone()
    b = e2.reset().clone()
    assert torch.equal(a, b)
    a2 = e1.reset().clone()  # unseeded: continues the PCG64 stream -> new maps
    assert not torch.equal(a, a2)
    assert torch.equal(a2, e2.reset())


def test_masked_reset(device):
    env = make_env(128, "mediumhard", 16, 9, device)
    base = env.reset().clone()
    st0 = env.get_state()
    mask = torch.zeros(128, dtype=torch.uint8, device=device)
    mask[::3] = 1
    out = env.reset(mask=mask).clone()
    st1 = env.get_state()
    keep = (mask == 0).cpu().numpy()
    assert torch.equal(out[mask == 0], base[mask == 0])
    assert (st1["walls"][keep] == st0["walls"][keep]).all()
    assert not (st1["walls"][~keep] == st0["walls"][~keep]).all()


def test_single_env_gym_api(device, golden):
    """MerlinEnv: the ScenarioCreator.create_env drop-in (uint8 frames, gym tuples)."""
    import oracle as O

    from merlin import ScenarioCreator

    env = ScenarioCreator().create_env("mediumhard")
    obs, info = env.reset(seed=777)
    assert obs.shape == (56, 56, 3) and obs.dtype == np.uint8 and info == {}
    codes, _, _, _, _ = O.batch_rollout(np.array([777], np.uint64), np.zeros((1, 1), np.int64))
    assert (obs == O.render(codes[0], golden("atlas")["atlas"])[0]).all()
    obs2, r, te, tr, _ = env.step(0)
    assert isinstance(r, float) and te is False and tr is False
    assert (obs2 == O.render(codes[1], golden("atlas")["atlas"])[0]).all()
    assert env.action_space.n == 3
    with pytest.raises(IndexError):
        env.step(3)


@pytest.mark.parametrize("diff,size", [("mediumhard", 16), ("hard", 22), ("hardest", 16)])
def test_full_observation_vs_state(device, diff, size):
    """merlin_env_full_obs (observation.fully_observable: FullyObsWrapper + ImgObsWrapper) equals the bit-row
    restatement of minigrid's Grid.encode (oracle/minigrid_literal.full_obs_from_state) on the state the env reports,
    after resets and random steps with auto-reset."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    from minigrid_literal import full_obs_from_state

    env = make_env(300, diff, size, 11, device)
    env.reset()
    g = torch.Generator(device=device).manual_seed(4)
    for k in range(12):
        if k:
            env.step(torch.randint(0, 3, (300,), device=device, generator=g))
        full = env.render_full().cpu().numpy()
        st = env.get_state()
        assert full.shape == (300, size, size, 3)
        for i in range(0, 300, 7):
            want = full_obs_from_state(st["walls"][i], st["agent_pos"][i], st["agent_dir"][i], st["goal_pos"][i], size)
            assert np.array_equal(full[i], want), (k, i)


def test_single_env_observation_modes(device, tmp_path):
    """The single env's observation options (scenario_creator.py:45-53): the full grid encoding, flattened or not,
    and the flattened RGB view; PPO takes a flattened observation down the reference's MLP path (src/ppo.py:38-41)."""
    from merlin import MerlinEnv
    from merlin.actor_critic import MLPActorCritic
    from merlin.ppo import PPO
    from merlin.scenario_creator import ScenarioCreator

    full = MerlinEnv("easy", device=device, fully_observable=True)
    obs, _ = full.reset(seed=5)
    assert obs.shape == (16, 16, 3) and obs.dtype == np.uint8 and full.observation_space.shape == (16, 16, 3)
    ax, ay = full.agent_pos
    assert obs[ax, ay, 0] == 10
    flat = MerlinEnv("easy", device=device, fully_observable=True, flatten=True)
    fobs, _ = flat.reset(seed=5)
    assert fobs.shape == (768,) and np.array_equal(fobs, obs.reshape(-1))
    o2, *_ = flat.step(2)
    o1, *_ = full.step(2)
    assert np.array_equal(o2, o1.reshape(-1))
    rgb = MerlinEnv("easy", device=device, flatten=True)
    robs, _ = rgb.reset(seed=5)
    assert robs.shape == (56 * 56 * 3,)
    p = tmp_path / "s.yaml"
    p.write_text("observation:\n  fully_observable: true\n  flatten: true\n"
                 "difficulties:\n  easy:\n    env_id: MERLIN-Easy-v0\n    params:\n      size: 16\n")
    env = ScenarioCreator(str(p)).create_env("easy")
    assert env.observation_space.shape == (768,)
    torch.manual_seed(0)
    agent = PPO(env, batch_size=64, minibatch_size=32, update_epochs=1, device=device)
    assert isinstance(agent.ac, MLPActorCritic) and agent.obs_shape == (768,)
    stats = agent.update(agent.collect_rollouts())
    assert all(np.isfinite(v) for v in stats.values())
