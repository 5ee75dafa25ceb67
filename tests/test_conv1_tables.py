"""CPU: the conv1-from-codes algebra.  P = einsum(W1, atlas/255) looked up at the 4
quarter-tile slots of every output position reproduces Conv2d(3,32,k8,s4) on the
rendered frames (fp32 tolerance), and autograd through the einsum gives conv1's dW.
The lookup here is a torch gather emulation of csrc/merlin_conv1.hip (the HIP kernels
are compared against this and against F.conv2d in tests/test_gpu_conv1.py)."""
import numpy as np
import torch
import torch.nn.functional as F


def emulate_lookup(P, b, codes49):
    """P [T,32,4,20], b [T,32], codes49 int64 [n,49] -> relu(z1) [T,n,32,13,13]."""
    n = codes49.shape[0]
    oy = torch.arange(13).view(13, 1).expand(13, 13)
    ox = torch.arange(13).view(1, 13).expand(13, 13)
    z = b[:, None, :, None, None].expand(-1, n, -1, 13, 13).clone()
    for dy in range(2):
        for dx in range(2):
            qr, qc = oy + dy, ox + dx
            cell = (qr // 2) * 7 + qc // 2  # [13,13]
            cls = codes49[:, cell.reshape(-1)].reshape(n, 13, 13)
            binv = cls * 4 + ((qr % 2) * 2 + (qc % 2))[None]
            slot = dy * 2 + dx
            tab = P[:, :, slot, :]  # [T,32,20]
            z = z + tab[:, None, :, :].expand(-1, n, -1, -1).gather(
                3, binv[None, :, None].expand(P.shape[0], n, 32, 13, 13).reshape(P.shape[0], n, 32, 169)
            ).reshape(P.shape[0], n, 32, 13, 13)
    return torch.relu(z)


def test_table_lookup_equals_conv2d(golden):
    import oracle as O

    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(3)
    ac = CNNActorCritic((56, 56, 3), 3)
    atlas = golden("atlas")["atlas"]
    ac._atlas = torch.from_numpy(atlas).permute(0, 3, 1, 2).float().contiguous() / 255.0
    rs = np.random.RandomState(2)
    codes = rs.randint(0, 5, size=(12, 49)).astype(np.uint8)
    frames = torch.from_numpy(O.render(codes, atlas).astype(np.float32)).permute(0, 3, 1, 2)
    P, b = ac.conv1_tables()
    got = emulate_lookup(P, b, torch.from_numpy(codes.astype(np.int64)))
    for t, tower in enumerate((ac.actor_extractor, ac.critic_extractor)):
        ref = torch.relu(F.conv2d(frames / 255.0, tower.network[0].weight, tower.network[0].bias, stride=4))
        torch.testing.assert_close(got[t], ref, rtol=1e-5, atol=1e-5)


def test_table_gradient_equals_conv_weight_gradient(golden):
    import oracle as O

    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(4)
    ac = CNNActorCritic((56, 56, 3), 3).double()
    atlas = golden("atlas")["atlas"]
    ac._atlas = torch.from_numpy(atlas).permute(0, 3, 1, 2).double().contiguous() / 255.0
    rs = np.random.RandomState(5)
    codes = rs.randint(0, 5, size=(6, 49)).astype(np.uint8)
    frames = torch.from_numpy(O.render(codes, atlas).astype(np.float64)).permute(0, 3, 1, 2)
    g = torch.randn(2, 6, 32, 13, 13, dtype=torch.float64)
    P, b = ac.conv1_tables()
    (emulate_lookup(P, b, torch.from_numpy(codes.astype(np.int64))) * g).sum().backward()
    dW = [ac.actor_extractor.network[0].weight.grad.clone(), ac.critic_extractor.network[0].weight.grad.clone()]
    dB = [ac.actor_extractor.network[0].bias.grad.clone(), ac.critic_extractor.network[0].bias.grad.clone()]
    ac.zero_grad()
    for t, tower in enumerate((ac.actor_extractor, ac.critic_extractor)):
        (torch.relu(F.conv2d(frames / 255.0, tower.network[0].weight, tower.network[0].bias, stride=4)) * g[t]).sum().backward()
        torch.testing.assert_close(dW[t], tower.network[0].weight.grad, rtol=1e-9, atol=1e-9)
        torch.testing.assert_close(dB[t], tower.network[0].bias.grad, rtol=1e-9, atol=1e-9)


def test_gemm_tower_layout_algebra(golden):
    """The GEMM formulation used by CNNActorCritic._forward_codes (K order (ky, kx, ci),
    W2t/W3t permutes, fc1 columns permuted to (p3, co)) equals the reference towers.
    F.unfold stands in for the HIP im2col kernels (checked on the GPU separately)."""
    import oracle as O

    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(6)
    ac = CNNActorCritic((56, 56, 3), 3).double()
    atlas = golden("atlas")["atlas"]
    rs = np.random.RandomState(7)
    codes = rs.randint(0, 5, size=(5, 49)).astype(np.uint8)
    x = torch.from_numpy(O.render(codes, atlas).astype(np.float64)).permute(0, 3, 1, 2) / 255.0
    n = x.shape[0]
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network

    def im2col(a, k, s):  # [n, C, H, W] -> [n*P, k*k*C] with K order (ky, kx, ci)
        C = a.shape[1]
        u = F.unfold(a, kernel_size=k, stride=s)  # [n, C*k*k, P] order (ci, ky, kx)
        P = u.shape[-1]
        return u.view(n, C, k * k, P).permute(0, 3, 2, 1).reshape(n * P, k * k * C)

    A2 = torch.stack([im2col(torch.relu(t[0](x)), 4, 2) for t in (ea, ec)])
    W2t = torch.stack([ea[2].weight, ec[2].weight]).permute(0, 3, 4, 2, 1).reshape(2, 512, 64)
    Z2 = torch.bmm(A2, W2t)
    b2 = torch.stack([ea[2].bias, ec[2].bias])
    a2 = torch.relu(Z2 + b2[:, None, :]).view(2, n, 5, 5, 64).permute(0, 1, 4, 2, 3)  # [2, n, 64, 5, 5]
    A3 = torch.stack([im2col(a2[t], 3, 1) for t in range(2)])
    W3t = torch.stack([ea[4].weight, ec[4].weight]).permute(0, 3, 4, 2, 1).reshape(2, 576, 64)
    b3 = torch.stack([ea[4].bias, ec[4].bias]).unsqueeze(1)
    a3 = torch.relu(torch.baddbmm(b3, A3, W3t)).view(2, n, 576)
    fa, fc = ac.actor[0], ac.critic[0]
    W4 = torch.stack([fa.weight, fc.weight])
    W4p = W4.view(2, 512, 64, 9).transpose(2, 3).reshape(2, 512, 576)
    h = torch.relu(torch.baddbmm(torch.stack([fa.bias, fc.bias]).unsqueeze(1), a3, W4p.transpose(1, 2)))
    logits = F.linear(h[0], ac.actor[2].weight, ac.actor[2].bias)
    value = F.linear(h[1], ac.critic[2].weight, ac.critic[2].bias).squeeze(-1)
    ref_logits = ac.actor(ac.actor_extractor(x, prescaled=True))
    ref_value = ac.critic(ac.critic_extractor(x, prescaled=True)).squeeze(-1)
    torch.testing.assert_close(logits, ref_logits, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(value, ref_value, rtol=1e-10, atol=1e-10)
