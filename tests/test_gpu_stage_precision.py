"""GPU: the fast step's conv tables (csrc/merlin_stage.hip: T2 from conv1 / conv2's weights and its adjoint down to
dW1 / db1 / dW2) are at least as accurate as the torch formulation they replace (CNNActorCritic.conv2_tables_from +
autograd in fp32, src/actor_critic.py:9-14 conv1 / conv2), both measured against the same formulation in float64,
on the model's initial weights (seed 777) and on random ones.  Norm-wise and max-element relative errors."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, r):
    a, r = a.double(), r.double()
    return float((a - r).norm() / r.norm().clamp_min(1e-300)), float((a - r).abs().max() / r.abs().max())


@pytest.mark.parametrize("weights", ["init", "random"])
def test_stage_tables_no_less_accurate_than_torch(device, weights):
    from merlin import CNNActorCritic
    from merlin import _native as nat

    torch.manual_seed(777)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    g = torch.Generator(device=device).manual_seed(1)
    if weights == "init":
        W1, b1, W2 = (torch.stack([ea[0].weight, ec[0].weight]).detach(),
                      torch.stack([ea[0].bias, ec[0].bias]).detach(), torch.stack([ea[2].weight, ec[2].weight]).detach())
    else:
        W1 = torch.randn(2, 32, 3, 8, 8, device=device, generator=g) * 0.2
        b1 = torch.randn(2, 32, device=device, generator=g) * 0.1
        W2 = torch.randn(2, 64, 32, 4, 4, device=device, generator=g) * 0.1
    dT2 = torch.randn(2, nat.LUT2_ROWS, 64, device=device, generator=g)
    atlas, idx, koff, kv = ac.stage_consts(device)
    res = {}
    for dt in (torch.float64, torch.float32):
        leaves = [x.to(dt).clone().requires_grad_() for x in (W1, b1, W2)]
        ac._lut2_gather = None
        T2 = ac.conv2_tables_from(*leaves)
        res[dt] = (T2.detach(),) + torch.autograd.grad(T2, leaves, grad_outputs=dT2.to(dt))
    HT, T2h = nat.stage_tables_fwd(W1.contiguous(), b1.contiguous(), W2.contiguous(), atlas, idx)
    hip = (T2h,) + tuple(nat.stage_tables_bwd(W2.contiguous(), HT, dT2.contiguous(), atlas, koff, kv))
    for name, h, t, r in zip(("T2", "dW1", "db1", "dW2"), hip, res[torch.float32], res[torch.float64]):
        eh, et = _rel(h, r), _rel(t, r)
        print(f"[{weights}] {name}: hip {eh[0]:.2e} / {eh[1]:.2e}  torch {et[0]:.2e} / {et[1]:.2e}")
        # no further from float64 than torch's fp32 (a float32 rounding's slack for ties at that level)
        assert eh[0] <= et[0] + 3e-8 and eh[1] <= et[1] + 6e-8, (name, eh, et)
