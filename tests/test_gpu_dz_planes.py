"""GPU: fc1's operands as h3 planes straight out of their producers (round 5; merlin/fast_step.py DZ_PLANES,
A3_PLANES): dz from the heads' backward, a3 from conv3's representatives.

merlin_tower_head_bwd_planes scales dz's planes by a bound on max |dz| known before the pass -- max over k of
sum_j max|dlogits[:, j]| |Wa[j][k]| (critic: max|dvalue| |wc[k]|), the loss's maxima from merlin_ppo_loss_absmax --
so it writes them in its one pass over h.  Checked here: the bound is >= max |dz| and equals its definition; the
planes are exactly h3_split(dz, bound); the other outputs are unchanged bit for bit; the input gradient over both
operands' planes (merlin_h3_gemm_nt_planes, LDS-DMA) and the weight gradient staging dz's planes as copies
(merlin_h3_gemm_tn_gather_planes_a) give the same bits as the fp32-operand GEMMs with the same scale; and one
optimizer step on the fast path with and without the planes agrees to fp32 level.  conv3's representatives likewise
(merlin_tower_window_conv3_planes, scaled by relu(b3 + the sum over taps of Q's column maxima) >= every Y3), with the
forward and the weight gradient over a3's planes giving the fp32-operand kernels' bits at the same scales."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _heads_case(device, n, A=3, seed=0):
    g = torch.Generator(device=device).manual_seed(seed)
    h = torch.relu(torch.randn(2, n, 512, device=device, generator=g))
    dlogits = torch.randn(n, A, device=device, generator=g) * 1e-5
    dlogits[: n // 7] *= 2.0 ** -20  # rows far below the max
    dvalue = torch.randn(n, device=device, generator=g) * 3e-6
    Wa = torch.randn(A, 512, device=device, generator=g) * 0.01
    Wc = torch.randn(1, 512, device=device, generator=g)
    gm = torch.zeros(9, dtype=torch.int32, device=device)
    gmf = gm.view(torch.float32)
    gmf[:A] = dlogits.abs().amax(0)
    gmf[8] = dvalue.abs().amax()
    return h, dlogits, dvalue, Wa, Wc, gm


@pytest.mark.parametrize("n,A", [(1, 3), (1000, 3), (20011, 3), (777, 7)])
def test_head_bwd_planes(device, n, A):
    from merlin import _native as nat

    h, dlogits, dvalue, Wa, Wc, gm = _heads_case(device, n, A, seed=n + A)
    dz, db, dwa, dwc = nat.head_bwd(h, dlogits, dvalue, Wa, Wc)
    bound = torch.zeros(2, dtype=torch.int32, device=device)
    P, db2, dwa2, dwc2 = nat.head_bwd(h, dlogits, dvalue, Wa, Wc, amax=bound, grad_absmax=gm)
    assert torch.equal(db2, db) and torch.equal(dwa2, dwa) and torch.equal(dwc2, dwc)
    bf = bound.view(torch.float32)
    assert (bf >= dz.abs().amax(dim=(1, 2))).all()
    D = gm.view(torch.float32)
    want = torch.stack([(D[:A, None] * Wa.abs()).sum(0).amax(), (D[8] * Wc.abs().view(-1)).amax()])
    torch.testing.assert_close(bf, want, rtol=1e-6, atol=0)
    assert torch.equal(P, nat.h3_split(dz, bound))


@pytest.mark.parametrize("M", [1, 4099, 111111])
def test_gemm_nt_planes_equals_fp32_operand_gemm(device, M):
    """The input gradient dz @ W4 (N = 576, K = 512) over dz's planes (cfg 62) == the fp32-operand kernel with the
    same scale, bit for bit (the same products in the same order); ragged M."""
    from merlin import _native as nat

    h, dlogits, dvalue, Wa, Wc, gm = _heads_case(device, M, seed=M)
    dz, _, _, _ = nat.head_bwd(h, dlogits, dvalue, Wa, Wc)
    bound = torch.zeros(2, dtype=torch.int32, device=device)
    P, _, _, _ = nat.head_bwd(h, dlogits, dvalue, Wa, Wc, amax=bound, grad_absmax=gm)
    g = torch.Generator(device=device).manual_seed(5)
    W4t = torch.randn(2, 576, 512, device=device, generator=g) * 0.04
    amW = nat.h3_amax(W4t)
    Wp = nat.h3_split(W4t, amW)
    ref = nat.h3_gemm_nt(dz, bound, Wp, amW, cfg=11)
    got = nat.h3_gemm_nt_planes(P, bound, Wp, amW, cfg=62)
    assert torch.equal(got, ref)
    # and within the fp32 GEMM's accuracy of the float64 product (bound-scaled planes: test_gpu_h3's error model)
    C64 = torch.bmm(dz.double(), W4t.double().transpose(1, 2))
    den = torch.bmm(dz.abs().double(), W4t.abs().double().transpose(1, 2)).clamp_min(1e-300)
    tol = max(float(((torch.bmm(dz, W4t.transpose(1, 2)).double() - C64).abs() / den).max()), 2.0 ** -21)
    tmax = dz.abs().amax(dim=(1, 2), keepdim=True).double()
    absb = W4t.abs().double().sum(dim=2).unsqueeze(1)
    assert ((got.double() - C64).abs() <= tol * den + 2.0 ** -49 * tmax * absb).all()


@pytest.mark.parametrize("Kd,splits", [(3001, 32), (40000, 32), (257, 1)])
def test_gemm_tn_gather_planes_a(device, Kd, splits):
    """The weight gradient dz^T a3 with dz as planes and a3 gathered through a row map == the fp32-dz kernel with
    the same scale, bit for bit."""
    from merlin import _native as nat

    h, dlogits, dvalue, Wa, Wc, gm = _heads_case(device, Kd, seed=Kd + 1)
    dz, _, _, _ = nat.head_bwd(h, dlogits, dvalue, Wa, Wc)
    bound = torch.zeros(2, dtype=torch.int32, device=device)
    P, _, _, _ = nat.head_bwd(h, dlogits, dvalue, Wa, Wc, amax=bound, grad_absmax=gm)
    g = torch.Generator(device=device).manual_seed(Kd)
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    nc = Kd * 576 // 64
    rows = torch.randint(0, nc, (nc,), device=device, generator=g, dtype=torch.int32)
    am3 = nat.h3_amax(a3)
    ref = nat.h3_gemm_tn(dz, bound, a3, am3, splits=splits, rows=rows)
    got = nat.h3_gemm_tn(P, bound, a3, am3, splits=splits, rows=rows)
    assert torch.equal(got, ref)


def test_fast_step_dz_planes_close(device, monkeypatch):
    """One update on the fast step with dz as bound-scaled planes against the same update with fp32 dz: the first
    optimizer step's gradient of every parameter to fp32 level (1e-5 of its norm), the update statistics to 1e-4."""
    from merlin import MerlinVecEnv
    from merlin import fast_step
    from merlin.ppo import PPO

    def run(planes):
        monkeypatch.setattr(fast_step, "DZ_PLANES", planes)
        env = MerlinVecEnv(256, "mediumhard", seed=5, device=device)
        torch.manual_seed(3)
        agent = PPO(env, lr=1e-3, batch_size=256 * 64, minibatch_size=256 * 16, update_epochs=2, ent_coef=0.05,
                    device=device)
        grads = []
        ca = agent._clip_adam
        orig = ca.step

        def step():
            if not grads:
                grads.extend(p.grad.detach().clone() for p in agent.ac.parameters())
            return orig()

        ca.step = step
        stats = agent.update(agent.collect_rollouts())
        torch.cuda.synchronize()
        return agent, stats, grads

    a0, s0, g0 = run(False)
    a1, s1, g1 = run(True)
    for k in s0:
        assert abs(s0[k] - s1[k]) <= 1e-4 * max(1.0, abs(s0[k])), k
    for (k, _), x, y in zip(a0.ac.named_parameters(), g0, g1):
        rel = float((x - y).norm() / x.norm().clamp_min(1e-30))
        assert rel <= 1e-5, (k, rel)


def _window_case(device):
    from test_gpu_windows import _plan

    codes, plan = _plan(device)
    g = torch.Generator(device=device).manual_seed(21)
    perm = torch.randperm(codes.shape[0], device=device, generator=g)
    mb = plan.update_minibatches([perm], 3000, bulk=True)[0][0]
    Q = torch.randn(2, plan.num_windows, 576, device=device, generator=g) * 0.3
    b3 = torch.randn(2, 64, device=device, generator=g) * 0.1
    return plan, mb, Q, b3


def test_window_conv3_planes(device):
    """conv3's representatives written as h3 planes (merlin_tower_window_conv3_planes): the bound from Q's column
    maxima is >= every Y3 value and equals its definition; every representative row's planes are exactly h3_split of
    the fp32 row with that bound; the mask words are the fp32 kernel's; the workspace is left zero (two calls agree)."""
    from merlin import _native as nat

    plan, mb, Q, b3 = _window_case(device)
    n = int(mb.groups.numel())
    rr = mb.rep_row.long()
    reps = rr == torch.arange(n * 9, device=device)
    Y0, m0 = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True)
    bound = torch.zeros(2, dtype=torch.int32, device=device)
    P, m1 = nat.window_conv3_planes(Q, plan.wid, mb.groups, b3, mb.rep_row, bound)
    bf = bound.view(torch.float32)
    assert (bf >= Y0.view(2, -1).amax(1)).all()
    cmax = Q.view(2, -1, 9, 64).amax(1)  # [2, 9, 64]
    acc = cmax[:, 0]
    for tap in range(1, 9):
        acc = acc + cmax[:, tap]
    assert torch.equal(bf, torch.relu(acc + b3).amax(1))
    ref = nat.h3_split(Y0, bound)
    assert torch.equal(P[:, reps], ref[:, reps]) and torch.equal(m1[:, reps], m0[:, reps])
    bound2 = torch.zeros(2, dtype=torch.int32, device=device)
    P2, _ = nat.window_conv3_planes(Q, plan.wid, mb.groups, b3, mb.rep_row, bound2)
    assert torch.equal(bound2, bound) and torch.equal(P2[:, reps], P[:, reps])


def test_forward_and_wgrad_over_a3_planes(device):
    """The forward with the heads over a3's gathered planes (merlin_h3_gemm_nt_heads_planes) and the weight gradient
    over both operands' planes (merlin_h3_gemm_tn_gather_planes) == the fp32-operand kernels with the same scales,
    bit for bit."""
    from merlin import _native as nat

    plan, mb, Q, b3 = _window_case(device)
    n = int(mb.groups.numel())
    bound = torch.zeros(2, dtype=torch.int32, device=device)
    P, _ = nat.window_conv3_planes(Q, plan.wid, mb.groups, b3, mb.rep_row, bound)
    Y0, _ = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True)
    a3 = Y0.view(2, n, 576)
    a3p = P.view(2, n, 1152)
    g = torch.Generator(device=device).manual_seed(4)
    W4 = torch.randn(2, 512, 576, device=device, generator=g) * 0.04
    amW = nat.h3_amax(W4)
    P4 = nat.h3_split(W4, amW)
    b4 = torch.randn(2, 512, device=device, generator=g) * 0.1
    Wa = torch.randn(3, 512, device=device, generator=g) * 0.01
    Wc = torch.randn(1, 512, device=device, generator=g)
    h0, l0, v0 = nat.h3_gemm_nt_heads(a3, bound, P4, amW, b4, Wa, Wc, cfg=13, rows=mb.rep_row)
    h1, l1, v1 = nat.h3_gemm_nt_heads(a3p, bound, P4, amW, b4, Wa, Wc, cfg=13, rows=mb.rep_row)
    assert torch.equal(h1, h0) and torch.equal(l1, l0) and torch.equal(v1, v0)
    # the LDS-DMA forward over the gathered planes (cfg 60, k_h3_pqg): the same bits
    h2, l2, v2 = nat.h3_gemm_nt_heads(a3p, bound, P4, amW, b4, Wa, Wc, cfg=60, rows=mb.rep_row)
    assert torch.equal(h2, h0) and torch.equal(l2, l0) and torch.equal(v2, v0)
    _, dlogits, dvalue, _, _, _ = _heads_case(device, n, seed=n)
    gm = torch.zeros(9, dtype=torch.int32, device=device)
    gm.view(torch.float32)[:3] = dlogits.abs().amax(0)
    gm.view(torch.float32)[8] = dvalue.abs().amax()
    dz, _, _, _ = nat.head_bwd(h0, dlogits, dvalue, Wa, Wc)
    amz = torch.zeros(2, dtype=torch.int32, device=device)
    dzp, _, _, _ = nat.head_bwd(h0, dlogits, dvalue, Wa, Wc, amax=amz, grad_absmax=gm)
    ref = nat.h3_gemm_tn(dz, amz, a3, bound, rows=mb.rep_row)
    got = nat.h3_gemm_tn(dzp, amz, a3p, bound, rows=mb.rep_row)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("cfg", [20, 21])
@pytest.mark.parametrize("Kd,splits", [(1, 1), (31, 1), (257, 3), (3001, 32), (40000, 32), (111111, 32)])
def test_wgrad_dma_kernel_bitwise(device, Kd, splits, cfg):
    """The weight gradient's LDS-DMA TN kernel over both operands' planes (cfg 20 / 21, k_h3_tq on 128 / 64 x 192
    tiles: B's rows through a row map read from an LDS ring, rows past a split's end zero-sourced, the step count
    padded to the ring's period) == the register-staged TN on the same planes (cfg 0), bit for bit; split-K and
    ragged row counts."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(Kd + splits)
    dz = torch.randn(2, Kd, 512, device=device, generator=g) * 1e-6
    a3 = torch.relu(torch.randn(2, Kd, 576, device=device, generator=g))
    nc = Kd * 576 // 64
    rows = torch.randint(0, nc, (nc,), device=device, generator=g, dtype=torch.int32)
    amz, am3 = nat.h3_amax(dz), nat.h3_amax(a3)
    dzp, a3p = nat.h3_split(dz, amz), nat.h3_split(a3, am3)
    ref = nat.h3_gemm_tn(dzp, amz, a3p, am3, splits=splits, cfg=0, rows=rows)
    got = nat.h3_gemm_tn(dzp, amz, a3p, am3, splits=splits, cfg=cfg, rows=rows)
    assert torch.equal(got, ref)
