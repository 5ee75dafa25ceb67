"""Numerics of the three-plane GEMMs on cancellation-heavy sums (the update's fc1 weight gradient:
sum over ~111k rows whose terms nearly cancel).  Error relative to the float64 result's norm, for
the x6 kernels and for torch's fp32 GEMM, and for operands that are exact in bf16 (planes 1, 2 = 0:
isolates the matrix cores' accumulation)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def rel(C, C64):
    return float((C.double() - C64).norm() / C64.norm())


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Kd = 111_000
    a3 = torch.relu(torch.randn(2, Kd, 576, device=dev, generator=g))
    # dz: per-row sign flips with a tiny bias, so column sums cancel to ~1e-3 of sum |.|
    s = torch.where(torch.rand(2, Kd, 1, device=dev, generator=g) < 0.5005, 1.0, -1.0)
    dz = s * torch.rand(2, Kd, 512, device=dev, generator=g) * (torch.rand(2, Kd, 512, device=dev, generator=g) > 0.3)
    for name, (A, B) in {"fp32 operands": (dz, a3),
                         "bf16-exact operands": (dz.bfloat16().float(), a3.bfloat16().float())}.items():
        W64 = torch.bmm(A.double().transpose(1, 2), B.double())
        Wt = torch.bmm(A.transpose(1, 2), B)
        Wsk = sum(torch.bmm(A[:, i:i + 3500].transpose(1, 2), B[:, i:i + 3500]) for i in range(0, Kd, 3500))
        Ap, Bp = A.contiguous(), B.contiguous()
        print(f"[wgrad, {name}] |W|/sum|ab| = {float(W64.norm() / torch.bmm(A.abs().double().transpose(1, 2), B.abs().double()).norm()):.2e}")
        print(f"  torch fp32 bmm   rel err {rel(Wt, W64):.3e}")
        print(f"  torch split-K    rel err {rel(Wsk, W64):.3e}")
        for splits in (1, 8, 32):
            W = nat.x6_gemm_tn(Ap, Bp, splits=splits)
            print(f"  x6 tn splits {splits:2d} rel err {rel(W, W64):.3e}")
        # the same product through the NT kernel (transposed operands materialised)
        At = A.transpose(1, 2)[:, :, :Kd // 32 * 32].contiguous()
        Bt = nat.x6_split(B.transpose(1, 2)[:, :, :Kd // 32 * 32].contiguous())
        W64t = torch.bmm(A[:, :Kd // 32 * 32].double().transpose(1, 2), B[:, :Kd // 32 * 32].double())
        print(f"  x6 nt (K={Kd // 32 * 32})   rel err {rel(nat.x6_gemm_nt(At, Bt, cfg=1), W64t):.3e}")


if __name__ == "__main__":
    main()
