"""GPU: the tower GEMM epilogues (csrc/merlin_head.hip) against PyTorch fp32 references: the
in-place bias + ReLU, the ReLU backward with the bias gradient, and the fused heads backward
(fc1's ReLU mask, fc1's bias gradient, both heads' weight gradients) against autograd of
F.linear heads on relu(fc1); the column sums are fixed-order (bitwise run to run)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(1, 64), (77, 64), (5000, 512), (1000, 4), (40000, 64)])
def test_bias_relu_and_relu_bwd(device, rows, cols):
    from merlin import _native as nat

    torch.manual_seed(rows)
    z = torch.randn(2, rows, cols, device=device)
    b = torch.randn(2, cols, device=device)
    y = nat.bias_relu_(z.clone(), b)
    assert torch.equal(y, torch.relu(z + b[:, None]))
    dy = torch.randn_like(y)
    dz, db = nat.relu_bwd(y, dy)
    ref = torch.where(y > 0, dy, torch.zeros_like(dy))
    assert torch.equal(dz, ref)
    torch.testing.assert_close(db, ref.double().sum(1).float(), rtol=1e-5, atol=1e-3)
    assert torch.equal(db, nat.relu_bwd(y, dy)[1])


@pytest.mark.parametrize("n,A", [(1, 3), (333, 3), (20000, 3), (100, 8)])
def test_head_bwd_matches_autograd(device, n, A):
    from merlin import _native as nat

    torch.manual_seed(n + A)
    H = 512
    z = torch.randn(2, n, H, device=device, requires_grad=True)
    Wa = torch.randn(A, H, device=device, requires_grad=True)
    Wc = torch.randn(1, H, device=device, requires_grad=True)
    h = torch.relu(z)
    logits, value = F.linear(h[0], Wa), F.linear(h[1], Wc).squeeze(-1)
    gl, gv = torch.randn(n, A, device=device), torch.randn(n, device=device)
    ((logits * gl).sum() + (value * gv).sum()).backward()
    dz, db4, dWa, dWc = nat.head_bwd(h.detach(), gl, gv, Wa.detach(), Wc.detach())
    torch.testing.assert_close(dz, z.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(db4, z.grad.sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dWa, Wa.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dWc.view(1, H), Wc.grad, rtol=1e-4, atol=1e-3)
    assert torch.equal(dWa, nat.head_bwd(h.detach(), gl, gv, Wa.detach(), Wc.detach())[2])


@pytest.mark.parametrize("rows", [0, 1, 777, 6634])
def test_colsum_strided_rows(device, rows):
    """merlin_tower_colsum over strided rows (the conv3 bias gradient reads tap 0 of dQ [T, nw, 9, 64])
    against a float64 sum; fixed order: bitwise reproducible."""
    from merlin import _native as nat

    torch.manual_seed(rows)
    dQ = torch.randn(2, rows, 9, 64, device=device)
    x = dQ[:, :, 0]
    out = nat.colsum(x)
    torch.testing.assert_close(out.double(), x.double().sum(1), rtol=1e-5, atol=1e-5)
    assert torch.equal(out, nat.colsum(x))


@pytest.mark.parametrize("n,A,bias", [(1, 3, False), (333, 3, True), (70001, 3, False), (100, 8, True), (513, 1, True)])
def test_heads_fwd_matches_float64(device, n, A, bias):
    """merlin_tower_heads_fwd (both heads in one pass over h) against float64 F.linear: within float32
    summation error of the 512-term dot products, and the same bits on every call."""
    from merlin import _native as nat

    torch.manual_seed(n + A)
    h = torch.relu(torch.randn(2, n, 512, device=device))
    wa = torch.randn(A, 512, device=device) / 512 ** 0.5
    wc = torch.randn(1, 512, device=device) / 512 ** 0.5
    ba = torch.randn(A, device=device) if bias else None
    bc = torch.randn(1, device=device) if bias else None
    logits, value = nat.heads_fwd(h, wa, wc, ba, bc)
    rl = F.linear(h[0].double(), wa.double(), None if ba is None else ba.double())
    rv = F.linear(h[1].double(), wc.double(), None if bc is None else bc.double()).squeeze(-1)
    mag_l = F.linear(h[0].double().abs(), wa.double().abs()) + (0 if ba is None else ba.double().abs())
    mag_v = F.linear(h[1].double().abs(), wc.double().abs()).squeeze(-1) + (0 if bc is None else bc.double().abs())
    assert ((logits.double() - rl).abs() <= 1e-6 * mag_l + 1e-7).all()
    assert ((value.double() - rv).abs() <= 1e-6 * mag_v + 1e-7).all()
    l2, v2 = nat.heads_fwd(h, wa, wc, ba, bc)
    assert torch.equal(logits, l2) and torch.equal(value, v2)
