"""Probe: one h3 NT GEMM configuration at the update's shape, `reps` launches (for rocprofv3 --pmc passes).
    python scripts/probe_gemm_one.py <cfg> [reps] [planes 0/1] [U]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def main():
    cfg = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    planes = len(sys.argv) > 3 and sys.argv[3] == "1"
    U = int(sys.argv[4]) if len(sys.argv) > 4 else 111000
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
    W = torch.randn(2, 512, 576, device=dev, generator=g) / 24
    b = torch.zeros(2, 512, device=dev)
    amW = nat.h3_amax(W)
    Hp = nat.h3_split(W, amW)
    am3 = nat.h3_amax(a3)
    A = nat.h3_split(a3, am3).view(torch.float32) if planes else a3
    out = torch.empty(2, U, 512, device=dev)
    for _ in range(reps):
        nat.h3_gemm_nt(A, am3, Hp, amW, bias=b, cfg=cfg, out=out)
    torch.cuda.synchronize()
    print("done", cfg, reps, planes, flush=True)


if __name__ == "__main__":
    main()
