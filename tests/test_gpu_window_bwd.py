"""GPU: the window GEMM's backward and forward (csrc/merlin_winbwd.hip, merlin_window_gemm_bwd / _fwd; the
conv3-per-window part of src/actor_critic.py:13 in merlin/fast_step.py): da2w = [a2w > 0] * dQ W3r^T, db2 = its column sums,
dW3r = a2w^T dQ, against float64 products of the same fp32 operands.  Each output's error relative to the sum of
|products| may be no larger than torch's own fp32 GEMM's on the same operands (floor: one fp32 product, 2^-23); the
mask is exact; two calls give the same bits.  Window counts: one window, tile edges (31 / 32 / 33), split edges
(255 / 256 / 257) and the update's ~6.6k, one and two towers."""
import pytest
import torch

pytestmark = pytest.mark.gpu

FLOOR = 2.0 ** -23


def _err(C, C64, den):
    return float(((C.double() - C64).abs() / den.clamp_min(1e-300)).max())


@pytest.mark.parametrize("T,nw", [(2, 1), (2, 31), (1, 32), (2, 33), (2, 255), (1, 256), (2, 257), (2, 6571)])
def test_window_gemm_bwd_vs_float64(device, T, nw):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(nw + T)
    a2w = torch.relu(torch.randn(T, nw, 64, device=device, generator=g))
    W3r = torch.randn(T, 64, 576, device=device, generator=g) * 0.05
    dQ = torch.randn(T, nw, 576, device=device, generator=g) * 1e-3
    dQ[:, ::7] *= 1e-4  # rows of very different scales
    db3 = torch.empty(T, 64, device=device)
    da2w, db2, dW3r = nat.window_gemm_bwd(a2w, dQ, W3r, out_db3=db3)
    torch.cuda.synchronize()
    # db3: the tap-0 columns' sums (conv3's bias gradient)
    t64 = dQ[:, :, :64].double().sum(1)
    tden = dQ[:, :, :64].abs().double().sum(1)
    assert _err(db3, t64, tden) <= nw * 2.0 ** -24 + FLOOR
    mask = a2w > 0
    assert torch.equal(da2w[~mask], torch.zeros_like(da2w[~mask]))
    # input gradient (unmasked entries)
    P64 = torch.bmm(dQ.double(), W3r.double().transpose(1, 2))
    den = torch.bmm(dQ.abs().double(), W3r.abs().double().transpose(1, 2))
    Pf = torch.bmm(dQ, W3r.transpose(1, 2))
    tol = max(_err(Pf[mask], P64[mask], den[mask]), FLOOR)
    assert _err(da2w[mask], P64[mask], den[mask]) <= 2 * tol
    # db2: column sums of the masked input gradient
    D64 = torch.where(mask, P64, torch.zeros_like(P64))
    b64 = D64.sum(1)
    bden = torch.where(mask, den, torch.zeros_like(den)).sum(1)
    assert _err(db2, b64, bden) <= 4 * tol + nw * 2.0 ** -24
    # weight gradient
    W64 = torch.bmm(a2w.double().transpose(1, 2), dQ.double())
    wden = torch.bmm(a2w.abs().double().transpose(1, 2), dQ.abs().double())
    Wf = torch.bmm(a2w.transpose(1, 2), dQ)
    wtol = max(_err(Wf, W64, wden), FLOOR)
    assert _err(dW3r, W64, wden) <= 2 * wtol + 2.0 ** -22
    # fixed order: the same bits again
    db3b = torch.empty_like(db3)
    again = nat.window_gemm_bwd(a2w, dQ, W3r, out_db3=db3b)
    assert all(torch.equal(x, y) for x, y in zip(again + (db3b,), (da2w, db2, dW3r, db3)))
    # without db3: the same three outputs
    assert all(torch.equal(x, y) for x, y in zip(nat.window_gemm_bwd(a2w, dQ, W3r), (da2w, db2, dW3r)))


@pytest.mark.parametrize("T,nw", [(2, 1), (2, 33), (1, 256), (2, 6571)])
def test_window_gemm_fwd_vs_float64(device, T, nw):
    """Q = a2w W3r (merlin_window_gemm_fwd, the forward of the same window GEMM)."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(3 * nw + T)
    a2w = torch.relu(torch.randn(T, nw, 64, device=device, generator=g))
    a2w[:, ::5] *= 1e-5
    W3r = torch.randn(T, 64, 576, device=device, generator=g) * 0.05
    Q = nat.window_gemm_fwd(a2w, W3r)
    Q64 = torch.bmm(a2w.double(), W3r.double())
    den = torch.bmm(a2w.abs().double(), W3r.abs().double())
    tol = max(_err(torch.bmm(a2w, W3r), Q64, den), FLOOR)
    assert _err(Q, Q64, den) <= 2 * tol
    assert torch.equal(nat.window_gemm_fwd(a2w, W3r), Q)


def test_window_gemm_bwd_rejects_bad_arguments(device):
    from merlin import _native as nat

    L = nat.lib()
    assert L.merlin_window_gemm_bwd_work(0, 10) == -1 and L.merlin_window_gemm_bwd_work(2, 0) == -1
    a2w = torch.zeros(2, 40, 64, device=device)
    dQ = torch.zeros(2, 40, 576, device=device)
    W3r = torch.zeros(2, 64, 576, device=device)
    out = torch.empty(2, 40, 64, device=device)
    b, w = torch.empty(2, 64, device=device), torch.empty(2, 64, 576, device=device)
    work = torch.empty(4, device=device)
    rc = L.merlin_window_gemm_bwd(nat.ptr(a2w), nat.ptr(dQ), nat.ptr(W3r), 2, 40, nat.ptr(out), nat.ptr(b),
                                  nat.ptr(w), None, nat.ptr(work), 4, None)
    assert rc != 0 and b"work too small" in L.merlin_last_error()
