"""GPU: fc1's fp32 GEMMs on the bf16 matrix cores in exact three-plane form (csrc/merlin_gemm.hip).

The plane split must be lossless (x0 + x1 + x2 == x bit for bit); each GEMM is compared with a
float64 product of the same fp32 operands, and its error must be no larger than that of torch's
own fp32 GEMM (hipBLASLt) on the same operands, measured as max |C - C64| / sum_k |a_k b_k|
(tolerance written below: 2x hipBLASLt's error, floor 1e-6); on a cancellation-heavy weight
gradient (the update's: the result ~1e-2 of sum |a b|) the error relative to the result's norm must
not exceed hipBLASLt's own split-K product's.  Shapes: the update's fc1 (K = 576 / 512, N = 512 /
576) at row counts that are not tile multiples, both towers with their own operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL_FLOOR = 1e-6


def _err(C, C64, den):
    return float(((C.double() - C64).abs() / den.clamp_min(1e-300)).max())


def test_split_is_exact(device):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(1)
    x = torch.randn(1 << 18, device=device, generator=g)
    # exact wherever the third plane stays a normal number, |x| >= 2^-110 (below that the planes
    # lose bits under 2^-126 absolute: irrelevant at fc1's magnitudes)
    x = x * torch.exp2(torch.randint(-80, 100, x.shape, device=device, generator=g).float())
    x = torch.where(x.abs() < 2.0 ** -100, torch.ones_like(x), x)
    x[:6] = torch.tensor([0.0, -0.0, 1.0, -3.0e38, 1.1754944e-38, 0.1], device=device)
    P = nat.x6_split(x.view(-1, 128))
    assert P.shape == (x.numel() // 128, 384) and P.dtype == torch.int16
    assert torch.equal(nat.x6_join(P).view(-1), x)
    # plane 0 is the bf16 rounding of x (round to nearest)
    p0 = P.view(-1, 16, 3, 8)[:, :, 0].reshape(-1)
    assert torch.equal(p0.view(torch.bfloat16), x.to(torch.bfloat16))


@pytest.mark.parametrize("N,K,cfg", [(512, 576, 0), (576, 512, 1), (512, 576, 2), (576, 512, 3), (512, 576, 20),
                                     (576, 512, 22), (512, 576, 21), (576, 512, 23), (512, 576, 26),
                                     (576, 512, 27), (512, 576, 28), (512, 576, 24), (512, 576, 25)])
@pytest.mark.parametrize("M", [1, 777, 20011])
def test_gemm_nt_vs_float64(device, M, N, K, cfg):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(M + N)
    A = torch.relu(torch.randn(2, M, K, device=device, generator=g))
    B = torch.randn(2, N, K, device=device, generator=g) / K ** 0.5
    bias = torch.randn(2, N, device=device, generator=g)
    C64 = torch.bmm(A.double(), B.double().transpose(1, 2))
    den = torch.bmm(A.abs().double(), B.abs().double().transpose(1, 2))
    tol = max(2 * _err(torch.bmm(A, B.transpose(1, 2)), C64, den), TOL_FLOOR)
    Bp = nat.x6_split(B)
    C = nat.x6_gemm_nt(A, Bp, cfg=cfg)
    assert _err(C, C64, den) <= tol
    Cb = nat.x6_gemm_nt(A, Bp, bias=bias, cfg=cfg)
    assert torch.equal(Cb, torch.relu(C + bias.unsqueeze(1)))


@pytest.mark.parametrize("cfg", [0, 1, 2, 20, 21, 24, 25])
@pytest.mark.parametrize("Kd,splits", [(1, 1), (4093, 7), (40000, 32), (40000, 64)])
def test_gemm_tn_vs_float64(device, Kd, splits, cfg):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(Kd)
    dz = torch.randn(2, Kd, 512, device=device, generator=g) * (torch.rand(2, Kd, 512, device=device,
                                                                           generator=g) > 0.5)
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    den = torch.bmm(dz.abs().double().transpose(1, 2), a3.abs().double())
    tol = max(2 * _err(torch.bmm(dz.transpose(1, 2), a3), W64, den), TOL_FLOOR)
    W = nat.x6_gemm_tn(dz, a3, splits=splits, cfg=cfg)
    assert _err(W, W64, den) <= tol
    # fixed-order slab fold: bitwise reproducible
    assert torch.equal(W, nat.x6_gemm_tn(dz, a3, splits=splits, cfg=cfg))


@pytest.mark.parametrize("cfg", [0, 20, 21, 24, 25])
def test_gemm_tn_cancellation(device, cfg):
    """The update's weight gradient: ~1e5 rows whose terms nearly cancel (|W| ~ 1e-2 sum |a b|)."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(5)
    Kd = 60000
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    sgn = torch.where(torch.rand(2, Kd, 1, device=device, generator=g) < 0.5005, 1.0, -1.0)
    dz = sgn * torch.rand(2, Kd, 512, device=device, generator=g)
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    rel = lambda W: float((W.double() - W64).norm() / W64.norm())  # noqa: E731
    ref = rel(sum(torch.bmm(dz[:, i:i + 2000].transpose(1, 2), a3[:, i:i + 2000]) for i in range(0, Kd, 2000)))
    assert rel(nat.x6_gemm_tn(dz, a3, cfg=cfg)) <= ref


@pytest.mark.parametrize("impl", ["x6", "h3"])
def test_window_update_x6_matches_hipblaslt(device, impl):
    """One window-path forward + backward with fc1 on the plane-form GEMMs (x6: bf16 three-plane, h3: f16
    two-plane, csrc/merlin_h3.hip) vs the same with torch's fp32 GEMMs: outputs and every parameter gradient agree
    to fp32 GEMM accuracy."""
    from merlin import CNNActorCritic

    from test_gpu_windows import _plan

    codes, plan = _plan(device)
    torch.manual_seed(11)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    mb = plan.minibatch(torch.randperm(codes.shape[0], device=device)[:3000])
    outs, grads = {}, {}
    for which in (impl, "hipblaslt"):
        ac.fc1_impl = which
        ac.zero_grad()
        logits, value = ac.heads_windows(plan, mb)
        (logits.square().sum() + value.sum()).backward()
        outs[which] = (logits.detach().clone(), value.detach().clone())
        grads[which] = {k: p.grad.detach().clone() for k, p in ac.named_parameters()}
    for a, b in zip(outs[impl], outs["hipblaslt"]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    for k in grads[impl]:
        g1, g2 = grads[impl][k], grads["hipblaslt"][k]
        scale = float(g2.abs().max()) + 1e-12
        assert float((g1 - g2).abs().max()) <= 2e-5 * scale, k
