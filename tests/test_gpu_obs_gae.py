"""GPU parity: observation expansion (bit-exact vs the oracle render of the same codes)
and GAE / advantage normalisation (vs the reference's own outputs: gae_ref.npz,
tolerance 1e-5 as north_star states; the thread-per-env kernel keeps the reference's
fp32 op order and is checked bit-exact too)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def pack(codes_u8: np.ndarray) -> np.ndarray:
    n = codes_u8.shape[0]
    nib = np.zeros((n, 64), dtype=np.uint32)
    nib[:, :49] = codes_u8
    w = (nib.reshape(n, 8, 8) << (4 * np.arange(8, dtype=np.uint32))).sum(-1).astype(np.uint32)
    return w.view(np.int32)


@pytest.fixture(scope="module")
def codes_case():
    rs = np.random.RandomState(0)
    c = rs.randint(0, 5, size=(777, 49)).astype(np.uint8)
    c[:, 45] = 4
    return c


def test_expand_u8_matches_oracle_render(golden, oracle, device, codes_case):
    from merlin import _native as nat

    codes = torch.from_numpy(pack(codes_case)).to(device)
    out = nat.expand_obs_u8(codes).cpu().numpy()
    ref = oracle.render(codes_case, golden("atlas")["atlas"])
    assert (out == ref).all()


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
def test_expand_f32_layouts_and_scale(golden, oracle, device, codes_case, layout):
    from merlin import _native as nat

    codes = torch.from_numpy(pack(codes_case)).to(device)
    ref = oracle.render(codes_case, golden("atlas")["atlas"]).astype(np.float32)
    if layout == "nchw":
        ref = ref.transpose(0, 3, 1, 2)
    out = nat.expand_obs(codes, layout=layout).cpu().numpy()
    assert (out == ref).all()
    out = nat.expand_obs(codes, layout=layout, scale=1.0 / 255.0).cpu().numpy()
    assert (out == ref * np.float32(1.0 / 255.0)).all()


def test_expand_gather_by_index(golden, oracle, device, codes_case):
    from merlin import _native as nat

    codes = torch.from_numpy(pack(codes_case)).to(device)
    idx = torch.randperm(777, device=device)[:300]
    out = nat.expand_obs(codes, index=idx).cpu().numpy()
    ref = oracle.render(codes_case[idx.cpu().numpy()], golden("atlas")["atlas"]).astype(np.float32)
    assert (out == ref.transpose(0, 3, 1, 2)).all()


def test_expand_empty(device):
    from merlin import _native as nat

    codes = torch.zeros((0, 8), dtype=torch.int32, device=device)
    assert nat.expand_obs(codes).shape == (0, 3, 56, 56)


def _gae(device, r, v, d, lv, gamma=0.99, lam=0.95, stats=None):
    from merlin import _native as nat

    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(device)  # noqa: E731
    adv, ret = nat.gae(t(r), t(v), t(d), t(np.atleast_1d(lv)), gamma, lam, stats=stats)
    return adv.cpu().numpy(), ret.cpu().numpy()


def test_gae_single_env_vs_reference(golden, device):
    g = golden("gae_ref")
    for k in range(int(g["ncases"])):
        r, v, d, lv = g[f"c{k}_r"], g[f"c{k}_v"], g[f"c{k}_d"], g[f"c{k}_last"]
        adv, ret = _gae(device, r, v, d, lv)  # N=1: the wave-scan kernel
        np.testing.assert_allclose(adv, g[f"c{k}_adv"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ret, g[f"c{k}_ret"], rtol=1e-5, atol=1e-5)
        adv, ret = _gae(device, r, v, d, lv, gamma=0.995)  # compute_gae_standard (FOMAML gamma)
        np.testing.assert_allclose(adv, g[f"c{k}_adv995"], rtol=1e-5, atol=1e-5)


def test_gae_thread_kernel_bit_exact_with_reference_order(golden, oracle, device):
    """N > 256 takes the thread-per-env kernel: bit-exact with the reference op order."""
    g = golden("gae_ref")
    r1, v1, d1, l1 = g["c0_r"], g["c0_v"], g["c0_d"], g["c0_last"]
    T, N = r1.shape[0], 1024
    rs = np.random.RandomState(1)
    r = np.repeat(r1[:, None], N, 1) + rs.randn(T, N).astype(np.float32) * 0.01
    v = np.repeat(v1[:, None], N, 1) + rs.randn(T, N).astype(np.float32) * 0.1
    d = (rs.rand(T, N) < 0.01).astype(np.float32)
    d[:, 0] = d1
    r[:, 0], v[:, 0] = r1, v1
    lv = rs.randn(N).astype(np.float32)
    lv[0] = l1
    adv, ret = _gae(device, r, v, d, lv)
    assert (adv[:, 0] == g["c0_adv"]).all() and (ret[:, 0] == g["c0_ret"]).all()
    oadv, oret = oracle.gae_tn(r, v, d, lv)
    assert (adv == oadv).all() and (ret == oret).all()


@pytest.mark.parametrize("N", [1, 7, 256, 257, 4096])
def test_gae_and_normalisation_shapes(oracle, device, N):
    from merlin import _native as nat

    T = 256
    rs = np.random.RandomState(N)
    r = ((rs.rand(T, N) < 0.05) * rs.rand(T, N)).astype(np.float32)
    v = rs.randn(T, N).astype(np.float32)
    d = (rs.rand(T, N) < 0.02).astype(np.float32)
    lv = rs.randn(N).astype(np.float32)
    stats = torch.zeros(3, dtype=torch.float64, device=device)
    adv, ret = _gae(device, r, v, d, lv, stats=stats)
    oadv, oret = oracle.gae_tn(r, v, d, lv)
    np.testing.assert_allclose(adv, oadv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret, oret, rtol=1e-5, atol=1e-5)
    s = stats.cpu().numpy()
    assert s[0] == T * N
    # the moments are the f64 sums of the kernel's own f32 advantages
    np.testing.assert_allclose(s[1], adv.astype(np.float64).sum(), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(s[2], (adv.astype(np.float64) ** 2).sum(), rtol=1e-12)
    a = torch.from_numpy(adv).to(device)
    norm = nat.adv_normalize(a, stats).cpu().numpy()
    np.testing.assert_allclose(norm, oracle.adv_normalize(oadv), rtol=1e-5, atol=1e-5)
    # property at full size: normalised advantages have mean 0, unbiased std 1
    assert abs(norm.astype(np.float64).mean()) < 1e-5
    assert abs(norm.astype(np.float64).std(ddof=1) - 1.0) < 1e-4


def test_adv_normalisation_vs_reference(golden, device):
    from merlin import _native as nat

    g = golden("gae_ref")
    for k in range(int(g["ncases"])):
        stats = torch.zeros(3, dtype=torch.float64, device=device)
        _gae(device, g[f"c{k}_r"], g[f"c{k}_v"], g[f"c{k}_d"], g[f"c{k}_last"], stats=stats)
        a = torch.from_numpy(g[f"c{k}_adv"]).to(device)
        norm = nat.adv_normalize(a, stats).cpu().numpy()
        np.testing.assert_allclose(norm, g[f"c{k}_advnorm"], rtol=1e-5, atol=1e-5)
