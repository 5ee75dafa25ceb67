"""CPU: the oracle (oracle/) pinned against the golden vectors before it is trusted.

RNG: against numpy's own Generator(PCG64(SeedSequence)) draws (rng_numpy.npz).
Env: against the literal minigrid restatement run on numpy's real Generator
(env_maps.npz, env_trace.npz) -- minigrid itself is absent, so env parity is
"unpinned" w.r.t. minigrid; atlas: the survey's recorded values.
GAE: against the reference's own PPO.compute_gae / compute_gae_standard outputs.
"""
import numpy as np
import pytest


def test_seedsequence_pcg64_state(golden, oracle):
    g = golden("rng_numpy")
    for s, words in zip(g["seeds"], g["state_words"]):
        r = oracle.Rng(int(s))
        assert tuple(int(w) for w in words) == r.state_words()


def test_raw_stream(golden, oracle):
    g = golden("rng_numpy")
    for s, raw in zip(g["seeds"], g["raw64"]):
        r = oracle.Rng(int(s))
        assert [r.next64() for _ in range(raw.shape[0])] == [int(x) for x in raw]


def test_bounded_integers(golden, oracle):
    g = golden("rng_numpy")
    for s, lohi, out in zip(g["seeds"], g["int_lohi"], g["int_out"]):
        r = oracle.Rng(int(s))
        got = [r.integers(int(lo), int(hi)) for lo, hi in lohi]
        assert got == [int(x) for x in out]


def test_choice_without_replacement(golden, oracle):
    g = golden("rng_numpy")
    for s, args, outs in zip(g["seeds"], g["choice_args"], g["choice_out"]):
        r = oracle.Rng(int(s))
        for (pop, k), row in zip(args, outs):
            assert list(r.choice_noreplace(int(pop), int(k))) == [int(x) for x in row[:k]]


def test_rng_live_numpy(oracle):
    for seed in (3, 99, 2**33 + 1):
        gen = np.random.default_rng(seed)
        r = oracle.Rng(seed)
        for lo, hi in [(0, 16), (19, 40), (0, 4), (1, 15), (2, 6), (6, 13), (0, 2**31 - 1)]:
            for _ in range(50):
                assert int(gen.integers(lo, hi)) == r.integers(lo, hi)


MAP_KEYS = ["mediumhard_16", "hard_16", "hard_22", "easy_16", "medium_16", "hardest_16"]


@pytest.mark.parametrize("key", MAP_KEYS)
def test_maps(golden, oracle, key):
    g = golden("env_maps")
    diff, size = key.rsplit("_", 1)
    size = int(size)
    for s, cells, meta in zip(g[key + "_seeds"], g[key + "_cells"], g[key + "_meta"]):
        c, m = oracle.gen_map(size, diff, int(s))
        assert (c == cells).all(), (key, int(s))
        assert tuple(m[:5]) == tuple(meta), (key, int(s))


def test_retry_seeds_covered(oracle):
    # multi-attempt generations (the previous attempt's agent_pos blocks walls) are in the goldens
    assert oracle.gen_map(16, "mediumhard", 857)[1][5] == 3
    assert oracle.gen_map(22, "hard", 429)[1][5] == 2


@pytest.mark.parametrize("key", ["mediumhard_16", "hard_22", "easy_16"])
def test_traces(golden, oracle, key):
    g = golden("env_trace")
    diff, size = key.rsplit("_", 1)
    n, T, max_steps, base = (int(x) for x in g[key + "_cfg"])
    seeds = np.arange(base, base + n, dtype=np.uint64)
    codes, rew, term, trunc, agent = oracle.batch_rollout(seeds, g[key + "_actions"], size=int(size),
                                                          difficulty=diff, max_steps=max_steps)
    assert (codes == g[key + "_codes"]).all()
    assert (rew == g[key + "_reward"]).all()
    assert (term == g[key + "_term"]).all() and (trunc == g[key + "_trunc"]).all()
    assert (agent == g[key + "_agent"]).all()


def test_trace_goldens_cover_edges(golden):
    g = golden("env_trace")
    assert g["mediumhard_16_term"].sum() > 0 and g["mediumhard_16_trunc"].sum() > 0
    assert g["easy_16_term"].sum() > 0


def test_atlas_survey_values(golden):
    a = golden("atlas")["atlas"]
    R = a[..., 0]
    assert (R[0, 0, 0], R[0, 0, 1], R[0, 3, 3]) == (55, 33, 0)  # dark empty: corner, line, interior
    assert (R[1, 0, 0], R[1, 0, 1], R[1, 3, 3]) == (114, 99, 76)  # lit empty
    assert (R[2] == 146).all()  # lit wall
    assert (R[3] == 76).all() and (a[3, ..., 1] == 255).all()  # lit goal
    assert R[4, 3, 3] == 255 and R[4, 3, 0] == 99  # agent triangle pointing up


def test_gae_oracle_vs_reference(golden, oracle):
    g = golden("gae_ref")
    for k in range(int(g["ncases"])):
        r, v, d, lv = g[f"c{k}_r"], g[f"c{k}_v"], g[f"c{k}_d"], g[f"c{k}_last"]
        adv, ret = oracle.gae_tn(r, v, d, lv)
        assert (adv[:, 0] == g[f"c{k}_adv"]).all() and (ret[:, 0] == g[f"c{k}_ret"]).all()
        adv2, ret2 = oracle.gae_tn(r, v, d, lv, gamma=0.995)
        assert (adv2[:, 0] == g[f"c{k}_adv995"]).all() and (ret2[:, 0] == g[f"c{k}_ret995"]).all()
        np.testing.assert_allclose(oracle.adv_normalize(adv[:, 0]), g[f"c{k}_advnorm"], rtol=0, atol=1e-6)


def test_stuck_penalty_oracle_semantics(oracle):
    # spinning in place: counter increments per step without a move; >= 3 -> -0.1 each step
    seeds = np.array([5], dtype=np.uint64)
    acts = np.zeros((6, 1), dtype=np.int64)  # turn left 6x
    _, rew, _, _, _ = oracle.batch_rollout(seeds, acts, stuck=True)
    assert list(rew[:, 0]) == [0, 0, np.float32(-0.1), np.float32(-0.1), np.float32(-0.1), np.float32(-0.1)]
