"""GPU: conv1+conv2 as table lookups (csrc/merlin_conv2lut.hip) against the CPU-checked
restatement (tests/test_conv2_tables.py::lut2_rows) and against PyTorch's convolutions of
the rendered frames; the histogram backward against index_add; the whole codes-path tower
(CNNActorCritic.codes_impl "lut2") against the reference-structured frame path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_conv2_tables import lut2_rows

pytestmark = pytest.mark.gpu


def _codes(device, n, seed):
    from test_gpu_obs_gae import pack

    rs = np.random.RandomState(seed)
    c = rs.randint(0, 5, size=(n, 49)).astype(np.uint8)
    c[:, 45] = 4
    return c, torch.from_numpy(pack(c)).to(device)


def _model(device, seed):
    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(seed)
    return CNNActorCritic((56, 56, 3), 3).to(device)


@pytest.mark.parametrize("n,use_index", [(1, False), (3, True), (7, False), (333, True), (4097, False)])
def test_lut_forward_matches_emulation_and_conv(device, n, use_index):
    from merlin import _native as nat

    c49, codes = _codes(device, max(n, 50), seed=n)
    ac = _model(device, 31)
    idx = torch.randint(0, codes.shape[0], (n,), device=device) if use_index else None
    with torch.no_grad():
        T2 = ac.conv2_tables().contiguous()
        Z2 = nat.conv2_lut_fwd(codes if use_index else codes[:n], idx, T2)
        sel = idx.cpu().numpy() if use_index else np.arange(n)
        rows = torch.from_numpy(lut2_rows(c49[sel])).to(device)
        frames = nat.expand_obs(codes, index=idx, scale=1.0 / 255.0) if use_index else \
            nat.expand_obs(codes[:n], scale=1.0 / 255.0)
        for t, net in enumerate((ac.actor_extractor.network, ac.critic_extractor.network)):
            emu = T2[t][rows].sum(2).reshape(n * 25, 64)
            torch.testing.assert_close(Z2[t], emu, rtol=1e-5, atol=1e-5)
            ref = F.conv2d(torch.relu(net[0](frames)), net[2].weight, stride=2)
            torch.testing.assert_close(Z2[t], ref.permute(0, 2, 3, 1).reshape(n * 25, 64), rtol=1e-4, atol=1e-4)


def test_col2im_chunked_layout(device):
    from merlin import _native as nat

    n = 77
    dA3 = torch.randn(2, n * 9, 576, device=device)
    Z2 = torch.randn(2, n * 25, 64, device=device)
    b2 = torch.randn(2, 64, device=device)
    flat = nat.conv3_col2im_bwd(dA3, Z2, b2)
    ch, absmax = nat.conv3_col2im_bwd_chunked(dA3, Z2, b2)
    assert torch.equal(ch.permute(0, 2, 1, 3).reshape(2, n * 25, 64), flat)
    assert absmax.view(torch.float32).item() == flat.abs().max().item()


@pytest.mark.parametrize("n,use_index", [(1, False), (5, True), (300, True), (9000, False)])
def test_lut_histogram_matches_index_add(device, n, use_index):
    from merlin import _native as nat

    c49, codes = _codes(device, max(n, 64), seed=100 + n)
    idx = torch.randint(0, codes.shape[0], (n,), device=device) if use_index else None
    g = torch.randn(2, n * 25, 64, device=device)
    g[g.abs() < 0.3] = 0.0  # ReLU-masked zeros, as col2im3 produces
    dZ2c = g.view(2, n * 25, 16, 4).permute(0, 2, 1, 3).contiguous()
    dT = nat.conv2_lut_bwd(codes.index_select(0, idx) if use_index else codes, dZ2c)
    sel = idx.cpu().numpy() if use_index else np.arange(n)
    rows = torch.from_numpy(lut2_rows(c49[sel])).to(device).reshape(n * 25, 16)
    ref = torch.zeros(2, 2720, 64, dtype=torch.float64, device=device)
    mag = torch.zeros_like(ref)  # sum of |terms| per bin: the scale of fp32 summation error
    for k in range(16):
        for t in range(2):
            ref[t].index_add_(0, rows[:, k], g[t].double())
            mag[t].index_add_(0, rows[:, k], g[t].double().abs())
    err = (dT.double() - ref).abs()
    assert (err <= 1e-5 * mag + 1e-6).all(), (err / (mag + 1e-6)).max().item()


@pytest.mark.parametrize("impl", ["lut2", "gemm"])
def test_codes_tower_forward_and_grads_match_frames(device, impl):
    from merlin import _native as nat

    _, codes = _codes(device, 1500, seed=10)
    idx = torch.randint(0, 1500, (1024,), device=device)
    acts = torch.randint(0, 3, (1024,), device=device)
    ac = _model(device, 11)
    ac.codes_impl = impl

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
