"""Probe: accuracy of the conv1 / conv2 tables T2 and their weight gradients against float64, for the torch
formulation (CNNActorCritic.conv2_tables_from + autograd, fp32) and csrc/merlin_stage.hip (merlin_stage_tables_fwd
/ _bwd), on the model's own initial weights (seed 777) and on random ones.  Prints norm-wise and max relative errors.
    python scripts/probe_stage_precision.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import CNNActorCritic
from merlin import _native as nat


def rel(a, r):
    a, r = a.double(), r.double()
    return float((a - r).norm() / r.norm().clamp_min(1e-300)), float(((a - r).abs().max() / r.abs().max()))


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(777)
    ac = CNNActorCritic((56, 56, 3), 3).to(dev)
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    init = (torch.stack([ea[0].weight, ec[0].weight]).detach(), torch.stack([ea[0].bias, ec[0].bias]).detach(),
            torch.stack([ea[2].weight, ec[2].weight]).detach())
    g = torch.Generator(device=dev).manual_seed(1)
    rnd = (torch.randn(2, 32, 3, 8, 8, device=dev, generator=g) * 0.2, torch.randn(2, 32, device=dev, generator=g) * 0.1,
           torch.randn(2, 64, 32, 4, 4, device=dev, generator=g) * 0.1)
    atlas, idx, koff, kv = ac.stage_consts(dev)
    for name, (W1, b1, W2) in (("init", init), ("random", rnd)):
        dT2 = torch.randn(2, 2720, 64, device=dev, generator=g)
        leaves64 = [x.double().clone().requires_grad_() for x in (W1, b1, W2)]
        ac._lut2_gather = None
        T64 = ac.conv2_tables_from(*leaves64)
        g64 = torch.autograd.grad(T64, leaves64, grad_outputs=dT2.double())
        leaves32 = [x.float().clone().requires_grad_() for x in (W1, b1, W2)]
        ac._lut2_gather = None
        T32 = ac.conv2_tables_from(*leaves32)
        g32 = torch.autograd.grad(T32, leaves32, grad_outputs=dT2)
        HT, Th = nat.stage_tables_fwd(W1.contiguous(), b1.contiguous(), W2.contiguous(), atlas, idx)
        gh = nat.stage_tables_bwd(W2.contiguous(), HT, dT2.contiguous(), atlas, koff, kv)
        print(f"[{name}] T2    torch {rel(T32, T64)}  hip {rel(Th, T64)}", flush=True)
        for k, a, b, r in zip(("dW1", "db1", "dW2"), g32, gh, g64):
            print(f"[{name}] {k:5s} torch {rel(a, r)}  hip {rel(b, r)}", flush=True)


if __name__ == "__main__":
    main()
