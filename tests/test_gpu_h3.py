"""GPU: fc1's fp32 GEMMs on the f16 matrix cores in two-plane form (csrc/merlin_h3.hip).

Every operand is scaled by a per-tower power of two from its max |x| and used as two f16 planes; the planes must
reconstruct x' = x 2^e to 2^-23 |x'| (values within 2^26 of the tower max).  Each GEMM is compared with a float64
product of the same fp32 operands, and its error must be no larger than that of torch's own fp32 GEMM (hipBLASLt,
the f32 MFMA) on the same operands: max |C - C64| / sum_k |a_k b_k| (floor: one product's bound, 2^-21), and on the
update's
cancellation-heavy weight gradient the error relative to the result's norm.  Operand magnitudes include the
update's gradient scale (dz ~ 1e-7: only the per-tensor exponent keeps those inside the f16 range) and rows of
very different scales.  Shapes: the update's fc1 (K = 576 / 512, N = 512 / 576), row counts that are not tile
multiples, both towers with their own operands and scales."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# one product's own error bound: the two planes hold each scaled value to 2^-23, the dropped l_a l_b term is below
# 2^-22 |a b| -- together under 2^-21 |a b| (a K = 1 "GEMM" is a single product, exact in fp32); from K ~ 100 on the
# fp32 accumulation error of either GEMM is larger than this
FLOOR = 2.0 ** -21


def _err(C, C64, den):
    return float(((C.double() - C64).abs() / den.clamp_min(1e-300)).max())


def test_amax_and_split(device):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(3)
    x = torch.randn(2, 333, 576, device=device, generator=g)
    x[0] *= 1e-7
    x[1] *= 3e4
    am = nat.h3_amax(x)
    ref = x.abs().amax(dim=(1, 2))
    assert torch.equal(am.view(torch.float32), ref)
    P = nat.h3_split(x, am).view(torch.float16).view(2, 333, 72, 2, 8).float()
    e = 14 - torch.floor(torch.log2(ref))  # max |x| 2^e in [2^14, 2^15)
    xs = x * torch.exp2(e).view(2, 1, 1)
    assert float(xs.abs().amax()) < 2 ** 15 and float(xs.abs().amax()) >= 2 ** 14
    # the planes exactly: h = f16(x'), l = f16(2^11 (x' - h)) (round to nearest even; x' - h is exact in fp32)
    h = xs.view(2, 333, 72, 8).half()
    l = ((xs.view(2, 333, 72, 8) - h.float()) * 2048).half()
    assert torch.equal(P[..., 0, :].half(), h) and torch.equal(P[..., 1, :].half(), l)
    rec = (P[..., 0, :].double() + P[..., 1, :].double() / 2048).reshape(2, 333, 576)
    rel = ((rec - xs.double()).abs() / xs.double().abs().clamp_min(2 ** -12)).max()
    assert float(rel) <= 2 ** -23


def _operands(device, M, N, K, seed, scale_a=1.0, ragged=False):
    g = torch.Generator(device=device).manual_seed(seed)
    A = torch.relu(torch.randn(2, M, K, device=device, generator=g)) * scale_a
    if ragged:  # rows of very different magnitudes within one tensor
        A = A * torch.exp2(torch.randint(-12, 4, (2, M, 1), device=device, generator=g).float())
    B = torch.randn(2, N, K, device=device, generator=g) / K ** 0.5
    return A, B


@pytest.mark.parametrize("N,K,cfg", [(512, 576, 0), (576, 512, 1), (512, 576, 2), (576, 512, 2), (512, 576, 3),
                                     (512, 576, 10), (576, 512, 11), (512, 576, 12), (576, 512, 12), (512, 576, 13),
                                     (512, 576, 14),
                                     (512, 576, 20), (576, 512, 21), (512, 576, 30), (576, 512, 31)])
@pytest.mark.parametrize("M,scale_a,ragged", [(1, 1.0, False), (777, 1.0, False), (20011, 1.0, False),
                                              (20011, 1e-7, False), (9999, 1.0, True)])
def test_gemm_nt_vs_float64(device, M, N, K, cfg, scale_a, ragged):
    from merlin import _native as nat

    if N % {1: 192, 11: 192, 21: 192, 31: 192, 3: 256, 13: 256}.get(cfg, 128):
        pytest.skip("N not a multiple of the tile width")
    A, B = _operands(device, M, N, K, M + N + cfg, scale_a, ragged)
    bias = torch.randn(2, N, device=device)
    C64 = torch.bmm(A.double(), B.double().transpose(1, 2))
    den = torch.bmm(A.abs().double(), B.abs().double().transpose(1, 2))
    tol = max(_err(torch.bmm(A, B.transpose(1, 2)), C64, den), FLOOR)
    amA, amB = nat.h3_amax(A), nat.h3_amax(B)
    Bp = nat.h3_split(B, amB)
    C = nat.h3_gemm_nt(A, amA, Bp, amB, cfg=cfg)
    assert _err(C, C64, den) <= tol
    Cb = nat.h3_gemm_nt(A, amA, Bp, amB, bias=bias, cfg=cfg)
    assert torch.equal(Cb, torch.relu(C + bias.unsqueeze(1)))
    assert torch.equal(C, nat.h3_gemm_nt(A, amA, Bp, amB, cfg=cfg))  # fixed order: the same bits every call
    # every tile shape and staging path sums each output's products in the same order: the same bits
    assert torch.equal(C, nat.h3_gemm_nt(A, amA, Bp, amB, cfg=1 if N % 128 else 2))
    if cfg >= 20:
        return  # the DMA-staged kernel has no plane output
    P = torch.full((2, M, 2 * K), 0x5555, dtype=torch.int16, device=device)
    Cp = nat.h3_gemm_nt(A, amA, Bp, amB, cfg=cfg, planes_out=P)  # A's planes as a by-product: h3_split's exactly
    assert torch.equal(Cp, C) and torch.equal(P, nat.h3_split(A, amA))


@pytest.mark.parametrize("cfg", [0, 1, 10, 11])
@pytest.mark.parametrize("Kd,splits,scale", [(1, 1, 1.0), (4093, 7, 1.0), (40000, 32, 1.0), (40000, 32, 1e-7),
                                             (40000, 3, 1.0)])
def test_gemm_tn_vs_float64(device, Kd, splits, scale, cfg):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(Kd + cfg)
    dz = torch.randn(2, Kd, 512, device=device, generator=g) * (torch.rand(2, Kd, 512, device=device,
                                                                           generator=g) > 0.5) * scale
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    den = torch.bmm(dz.abs().double().transpose(1, 2), a3.abs().double())
    tol = max(_err(torch.bmm(dz.transpose(1, 2), a3), W64, den), FLOOR)
    amz, am3 = nat.h3_amax(dz), nat.h3_amax(a3)
    W = nat.h3_gemm_tn(dz, amz, a3, am3, splits=splits, cfg=cfg)
    assert _err(W, W64, den) <= tol
    assert torch.equal(W, nat.h3_gemm_tn(dz, amz, a3, am3, splits=splits, cfg=cfg))
    if cfg:  # every configuration sums each output's products in the same order
        assert torch.equal(W, nat.h3_gemm_tn(dz, amz, a3, am3, splits=splits, cfg=0))
    # over the operands' planes (what the fast step's NT GEMMs leave): the same images, the same bits
    Wq = nat.h3_gemm_tn(nat.h3_split(dz, amz), amz, nat.h3_split(a3, am3), am3, splits=splits, cfg=cfg % 10)
    assert torch.equal(Wq, W)


@pytest.mark.parametrize("cfg", [0, 1])
def test_gemm_tn_cancellation(device, cfg):
    """The update's weight gradient: ~1e5 rows whose terms nearly cancel (|W| ~ 1e-2 sum |a b|)."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(5)
    Kd = 60000
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    sgn = torch.where(torch.rand(2, Kd, 1, device=device, generator=g) < 0.5005, 1.0, -1.0)
    dz = sgn * torch.rand(2, Kd, 512, device=device, generator=g) * 1e-6
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    rel = lambda W: float((W.double() - W64).norm() / W64.norm())  # noqa: E731
    ref = rel(sum(torch.bmm(dz[:, i:i + 2000].transpose(1, 2), a3[:, i:i + 2000]) for i in range(0, Kd, 2000)))
    assert rel(nat.h3_gemm_tn(dz, nat.h3_amax(dz), a3, nat.h3_amax(a3), cfg=cfg)) <= ref


@pytest.mark.parametrize("cfg", [10, 11, 12, 13])
def test_gemm_nt_gather_rows_bitwise(device, cfg):
    """merlin_h3_gemm_nt_gather (A's rows read by 64-value chunks through a row map, as the update's forward reads
    conv3's patch representatives) == the same GEMM on the gathered matrix, bit for bit; tile-ragged row count,
    both towers, with and without the bias + ReLU epilogue."""
    from merlin import _native as nat

    M, K = 1000, 576
    N = 576 if cfg == 11 else 512
    A, B = _operands(device, M, N, K, 41 + cfg, ragged=True)
    g = torch.Generator(device=device).manual_seed(cfg)
    nc = M * K // 64
    rows = torch.randint(0, nc, (nc,), device=device, generator=g, dtype=torch.int32)
    keep = torch.rand(nc, device=device, generator=g) < 0.4  # some chunk rows read in place
    rows[keep] = torch.arange(nc, device=device, dtype=torch.int32)[keep]
    Ad = A.view(2, nc, 64)[:, rows.long()].reshape(2, M, K).contiguous()
    amA, amB = nat.h3_amax(Ad), nat.h3_amax(B)
    Bp = nat.h3_split(B, amB)
    bias = torch.randn(2, N, device=device, generator=g)
    for b in (None, bias):
        ref = nat.h3_gemm_nt(Ad, amA, Bp, amB, bias=b, cfg=cfg)
        got = nat.h3_gemm_nt(A, amA, Bp, amB, bias=b, cfg=cfg, rows=rows)
        assert torch.equal(got, ref)


@pytest.mark.parametrize("Kd,splits,cfg", [(3001, 32, 0), (40000, 32, 0), (700, 3, 1), (257, 1, 0)])
def test_gemm_tn_gather_rows_bitwise(device, Kd, splits, cfg):
    """merlin_h3_gemm_tn_gather (B's rows read by 64-column chunks through a row map: the weight gradient over
    conv3's patch representatives) == the same GEMM on the gathered matrix, bit for bit, split-K and ragged."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(Kd)
    M, N = 512, 576
    dz = torch.randn(2, Kd, M, device=device, generator=g) * 1e-7
    a3 = torch.relu(torch.randn(2, Kd, N, device=device, generator=g))
    nc = Kd * N // 64
    rows = torch.randint(0, nc, (nc,), device=device, generator=g, dtype=torch.int32)
    keep = torch.rand(nc, device=device, generator=g) < 0.4
    rows[keep] = torch.arange(nc, device=device, dtype=torch.int32)[keep]
    ad = a3.view(2, nc, 64)[:, rows.long()].reshape(2, Kd, N).contiguous()
    amz, am3 = nat.h3_amax(dz), nat.h3_amax(ad)
    ref = nat.h3_gemm_tn(dz, amz, ad, am3, splits=splits, cfg=cfg)
    got = nat.h3_gemm_tn(dz, amz, a3, am3, splits=splits, cfg=cfg, rows=rows)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("cfg,gather", [(13, False), (13, True), (12, False), (10, True), (14, False)])
def test_gemm_nt_heads_epilogue(device, cfg, gather):
    """merlin_h3_gemm_nt_heads (the policy / value heads folded into the forward GEMM's epilogue): h bit for bit as
    the plain bias + ReLU GEMM, logits / value against a float64 product of that h with the head weights (error no
    larger than merlin_heads_fwd's, which sums the same products in another order); ragged rows, 3 actions."""
    from merlin import _native as nat

    M, K, N = 1000, 576, 512
    A, B = _operands(device, M, N, K, 77 + cfg, ragged=True)
    g = torch.Generator(device=device).manual_seed(cfg)
    rows = None
    if gather:
        nc = M * K // 64
        rows = torch.randint(0, nc, (nc,), device=device, generator=g, dtype=torch.int32)
        A_eff = A.view(2, nc, 64)[:, rows.long()].reshape(2, M, K).contiguous()
    else:
        A_eff = A
    amA, amB = nat.h3_amax(A_eff), nat.h3_amax(B)
    Bp = nat.h3_split(B, amB)
    bias = torch.randn(2, N, device=device, generator=g)
    Wa = torch.randn(3, N, device=device, generator=g) / N ** 0.5
    Wc = torch.randn(1, N, device=device, generator=g) / N ** 0.5
    h_ref = nat.h3_gemm_nt(A_eff, amA, Bp, amB, bias=bias, cfg=cfg)
    h, logits, value = nat.h3_gemm_nt_heads(A, amA, Bp, amB, bias, Wa, Wc, cfg=cfg, rows=rows)
    assert torch.equal(h, h_ref)
    l64 = h_ref[0].double() @ Wa.double().T
    v64 = h_ref[1].double() @ Wc.double().view(-1)
    lf, vf = nat.heads_fwd(h_ref, Wa, Wc)
    den_l = h_ref[0].double().abs() @ Wa.double().abs().T
    den_v = h_ref[1].double().abs() @ Wc.double().abs().view(-1)
    assert _err(logits, l64, den_l) <= max(2 * _err(lf, l64, den_l), 2.0 ** -20)
    assert _err(value, v64, den_v) <= max(2 * _err(vf, v64, den_v), 2.0 ** -20)
    # fixed order: the same bits again
    h2, logits2, value2 = nat.h3_gemm_nt_heads(A, amA, Bp, amB, bias, Wa, Wc, cfg=cfg, rows=rows)
    assert torch.equal(logits2, logits) and torch.equal(value2, value) and torch.equal(h2, h)


@pytest.mark.parametrize("N,K,cfg", [(512, 576, 13), (576, 512, 11), (512, 576, 12)])
def test_gemm_nt_dynamic_range(device, N, K, cfg):
    """The h3 form's documented range (the bench line's dtype_note): rows spread over 2^-30 .. 2^3 of one
    scale.  Rows whose max lies within 2^26 of the tensor's max are held to the fp32 GEMM's own error (as above);
    below that the planes hold each value to 2^-50 of the tensor max, absolute, so those outputs' error stays under
    that absolute bound (x the row's sum of |b|) on top of the fp32 one."""
    from merlin import _native as nat

    M = 4099
    g = torch.Generator(device=device).manual_seed(N + cfg)
    A = torch.relu(torch.randn(2, M, K, device=device, generator=g))
    A = A * torch.exp2(torch.randint(-30, 4, (2, M, 1), device=device, generator=g).float())
    B = torch.randn(2, N, K, device=device, generator=g) / K ** 0.5
    C64 = torch.bmm(A.double(), B.double().transpose(1, 2))
    den = torch.bmm(A.abs().double(), B.abs().double().transpose(1, 2))
    amA, amB = nat.h3_amax(A), nat.h3_amax(B)
    C = nat.h3_gemm_nt(A, amA, nat.h3_split(B, amB), amB, cfg=cfg)
    Cf = torch.bmm(A, B.transpose(1, 2))
    tmax = A.abs().amax(dim=(1, 2), keepdim=True)  # [2, 1, 1]
    inr = (A.abs().amax(dim=2, keepdim=True) >= tmax * 2.0 ** -26).expand_as(C)  # [2, M, N]
    assert inr.any() and (~inr).any()
    tol = max(_err(Cf[inr], C64[inr], den[inr]), FLOOR)
    assert _err(C[inr], C64[inr], den[inr]) <= tol
    absb = B.abs().double().sum(dim=2).unsqueeze(1)  # [2, 1, N]: sum_k |b_nk|
    bound = tol * den + 2.0 ** -49 * tmax.double() * absb
    assert ((C.double() - C64).abs() <= bound)[~inr].all()


def test_gemm_tn_dynamic_range(device):
    """The weight gradient with dz rows spread over 2^-30 .. 2^0 of one scale (the update's per-sample gradient
    magnitudes vary that much): within the fp32 error plus the documented absolute bound for values below 2^-26 of
    the max."""
    from merlin import _native as nat

    Kd = 20000
    g = torch.Generator(device=device).manual_seed(11)
    dz = torch.randn(2, Kd, 512, device=device, generator=g) * 1e-6
    dz = dz * torch.exp2(torch.randint(-30, 1, (2, Kd, 1), device=device, generator=g).float())
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    den = torch.bmm(dz.abs().double().transpose(1, 2), a3.abs().double())
    tol = max(_err(torch.bmm(dz.transpose(1, 2), a3), W64, den), FLOOR)
    W = nat.h3_gemm_tn(dz, nat.h3_amax(dz), a3, nat.h3_amax(a3))
    zmax = dz.abs().amax(dim=(1, 2)).double().view(2, 1, 1)
    absa = a3.abs().double().sum(dim=1).unsqueeze(1)  # [2, 1, 576]
    assert ((W.double() - W64).abs() <= tol * den + 2.0 ** -49 * zmax * absa).all()


@pytest.mark.parametrize("N,K,cfg", [(576, 512, 62), (576, 512, 63), (576, 512, 66), (576, 512, 65), (576, 512, 69),
                                     (512, 576, 60), (512, 576, 68)])
@pytest.mark.parametrize("M,scale_a,ragged", [(777, 1.0, False), (20011, 1e-7, False), (9999, 1.0, True)])
def test_gemm_nt_planes_vs_float64(device, M, N, K, cfg, scale_a, ragged):
    """merlin_h3_gemm_nt_planes (both operands as planes, LDS-DMA staged, csrc/merlin_h3p.hip) at the update's shapes:
    the benched tiles (60 / 62), the 4-stage ring (63) and the product-major MFMA order (66) -- 62's products in 62's
    order, the same bits -- and the one-accumulator alternates (65 / 68 / 69: the lo planes rescaled in registers,
    another summation) all within torch's fp32 GEMM error against float64."""
    from merlin import _native as nat

    A, B = _operands(device, M, N, K, 7 * M + cfg, scale_a, ragged)
    C64 = torch.bmm(A.double(), B.double().transpose(1, 2))
    den = torch.bmm(A.abs().double(), B.abs().double().transpose(1, 2))
    tol = max(_err(torch.bmm(A, B.transpose(1, 2)), C64, den), FLOOR)
    amA, amB = nat.h3_amax(A), nat.h3_amax(B)
    Ap, Bp = nat.h3_split(A, amA), nat.h3_split(B, amB)
    C = nat.h3_gemm_nt_planes(Ap, amA, Bp, amB, cfg=cfg)
    assert _err(C, C64, den) <= tol
    assert torch.equal(C, nat.h3_gemm_nt_planes(Ap, amA, Bp, amB, cfg=cfg))  # fixed order: the same bits every call
    if cfg in (63, 66):
        assert torch.equal(C, nat.h3_gemm_nt_planes(Ap, amA, Bp, amB, cfg=62))
