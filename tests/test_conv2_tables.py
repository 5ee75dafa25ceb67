"""CPU: the conv1+conv2 table algebra of csrc/merlin_conv2lut.hip.

T2 = CNNActorCritic.conv2_tables() looked up at the 16 tap rows of every conv2 output
position reproduces Conv2d(32,64,k4,s2)(relu(Conv2d(3,32,k8,s4)(frame))) without the conv2
bias, and the histogram of dZ2 over those rows (what k_conv2_lut_hist computes), pushed
back through the table construction by autograd, gives the reference's conv1/conv2 weight
and bias gradients.  `lut2_rows` is a numpy restatement of the kernel's tap_rows(); the
HIP kernels are compared against it and against F.conv2d in tests/test_gpu_conv2lut.py."""
import numpy as np
import torch
import torch.nn.functional as F


def lut2_rows(cls49):
    """int [n, 49] tile classes -> int64 [n, 25, 16] table rows (tap = 4*ky + kx)."""
    c = np.asarray(cls49, dtype=np.int64).reshape(-1, 7, 7)
    n = c.shape[0]
    rows = np.zeros((n, 25, 16), dtype=np.int64)
    for py in range(5):
        for px in range(5):
            for ky in range(4):
                for kx in range(4):
                    r0, c0, j = py + (ky >> 1), px + (kx >> 1), 2 * (ky >> 1) + (kx >> 1)
                    w = lambda a, b: c[:, r0 + a, c0 + b]  # noqa: E731
                    if not ky & 1 and not kx & 1:
                        row = 4 * w(0, 0) + j
                    elif not ky & 1:
                        row = 20 + 4 * (5 * w(0, 0) + w(0, 1)) + j
                    elif not kx & 1:
                        row = 120 + 4 * (5 * w(0, 0) + w(1, 0)) + j
                    else:
                        row = 220 + 4 * (125 * w(0, 0) + 25 * w(0, 1) + 5 * w(1, 0) + w(1, 1)) + j
                    rows[:, py * 5 + px, ky * 4 + kx] = row
    return rows


def _model(seed, golden, dtype):
    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(seed)
    ac = CNNActorCritic((56, 56, 3), 3).to(dtype)
    atlas = golden("atlas")["atlas"]
    ac._atlas = torch.from_numpy(atlas).permute(0, 3, 1, 2).to(dtype).contiguous() / 255.0
    return ac, atlas


def test_rows_cover_every_table_row_type():
    from merlin.actor_critic import _LUT2_H1

    assert sum(4 * idx.shape[0] for _, idx in _LUT2_H1) == 2720
    rs = np.random.RandomState(0)
    rows = lut2_rows(rs.randint(0, 5, size=(4000, 49)))
    assert rows.min() >= 0 and rows.max() < 2720
    # tap j of a row is (row - base) % 4; type by tap parity
    for k in range(16):
        ky, kx = k >> 2, k & 3
        base = (0, 20, 120, 220)[2 * (ky & 1) + (kx & 1)]
        assert ((rows[:, :, k] - base) % 4 == 2 * (ky >> 1) + (kx >> 1)).all()


def test_table_lookup_equals_conv2_of_conv1(golden):
    import oracle as O

    ac, atlas = _model(21, golden, torch.float64)
    rs = np.random.RandomState(22)
    codes = rs.randint(0, 5, size=(9, 49)).astype(np.uint8)
    codes[:, 45] = 4
    x = torch.from_numpy(O.render(codes, atlas).astype(np.float64)).permute(0, 3, 1, 2) / 255.0
    T2 = ac.conv2_tables()
    rows = torch.from_numpy(lut2_rows(codes))
    for t, net in enumerate((ac.actor_extractor.network, ac.critic_extractor.network)):
        ref = F.conv2d(torch.relu(net[0](x)), net[2].weight, stride=2)  # [n, 64, 5, 5], no bias
        got = T2[t][rows].sum(2)  # [n, 25, 64]
        torch.testing.assert_close(got, ref.permute(0, 2, 3, 1).reshape(9, 25, 64), rtol=1e-10, atol=1e-10)


def test_histogram_gradient_equals_conv_gradients(golden):
    import oracle as O

    ac, atlas = _model(23, golden, torch.float64)
    rs = np.random.RandomState(24)
    n = 7
    codes = rs.randint(0, 5, size=(n, 49)).astype(np.uint8)
    x = torch.from_numpy(O.render(codes, atlas).astype(np.float64)).permute(0, 3, 1, 2) / 255.0
    g = torch.randn(2, n, 25, 64, dtype=torch.float64)  # dL/dZ2 (post-bias, pre-ReLU of conv2)
    rows = torch.from_numpy(lut2_rows(codes)).reshape(n * 25, 16)
    # the histogram k_conv2_lut_hist computes: dT[t][row] += dZ2[t][k, p] for each tap's row
    dT = torch.zeros(2, 2720, 64, dtype=torch.float64)
    for k in range(16):
        for t in range(2):
            dT[t].index_add_(0, rows[:, k], g[t].reshape(n * 25, 64))
    db2 = dT[:, 0:20:4, :].sum(1)
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    ac.conv2_tables().backward(dT)
    assert ea[2].bias.grad is None  # conv2 bias is not part of the tables
    mine = [[net[0].weight.grad.clone(), net[0].bias.grad.clone()] for net in (ea, ec)]
    mine = [mine[0], [ea[2].weight.grad.clone(), db2[0]], mine[1], [ec[2].weight.grad.clone(), db2[1]]]
    ac.zero_grad()
    for t, net in enumerate((ea, ec)):
        z2 = net[2](torch.relu(net[0](x)))
        (z2 * g[t].view(n, 5, 5, 64).permute(0, 3, 1, 2)).sum().backward()
    ref = [[m.weight.grad, m.bias.grad] for net in (ea, ec) for m in (net[0], net[2])]
    for a, b in zip(mine, ref):
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=1e-9, atol=1e-9)


def test_conv2_tables_function_matches_autograd_definition(golden):
    """_Conv2Tables (explicit forward/backward) == the per-parity-type autograd formulation:
    the table and the conv1 / conv2 weight and bias gradients, float64."""
    ac, _ = _model(5, golden, torch.float64)
    g = torch.Generator().manual_seed(3)
    dT = torch.randn(2, 2720, 64, dtype=torch.float64, generator=g)
    grads = []
    for fn in (ac.conv2_tables, ac._conv2_tables_autograd):
        ac.zero_grad(set_to_none=True)
        T = fn()
        T.backward(dT)
        grads.append([T.detach()] + [p.grad.clone() for p in (ac.actor_extractor.network[0].weight,
                                                             ac.critic_extractor.network[0].bias,
                                                             ac.actor_extractor.network[2].weight,
                                                             ac.critic_extractor.network[2].weight)])
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=1e-12, atol=1e-12)
