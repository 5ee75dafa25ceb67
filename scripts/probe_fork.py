"""Probe: is a side stream's first launch ordered after a fork (side.wait_stream(main)) whose last main-stream op
was one of the library's own launches (merlin._native, hipLaunchKernelGGL on torch's stream handle)?  Trial k, no
host synchronisation between trials: main runs a long library GEMM, then the library's x6_split of a tensor filled
with k into P; the side stream forks off main and reads P with the library's x6_join (or a torch op) into slot k.
    python scripts/probe_fork.py [trials]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    g0 = torch.Generator(device=dev).manual_seed(0)
    dz = torch.randn(2, 60000, 512, device=dev, generator=g0)
    a3 = torch.randn(2, 60000, 576, device=dev, generator=g0)
    amz, am3 = nat.h3_amax(dz), nat.h3_amax(a3)
    W = torch.empty(2, 512, 576, device=dev)
    vals = [torch.full((1 << 16,), float(k), device=dev) for k in range(trials + 1)]
    P = nat.x6_split(vals[0])
    R = torch.zeros(trials, device=dev)
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    for reader in ("library", "torch"):
        for last in ("library", "torch"):
            R.zero_()
            torch.cuda.synchronize()
            for k in range(1, trials + 1):
                nat.h3_gemm_tn(dz, amz, a3, am3, out=W)
                if last == "library":
                    nat.x6_split(vals[k], out=P)
                else:
                    P.view(-1, 3, 8)[:, 0].copy_(vals[k].view(-1, 8).to(torch.bfloat16).view(torch.int16))
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    if reader == "library":
                        R[k - 1].copy_(nat.x6_join(P)[-1])
                    else:
                        R[k - 1].copy_(P.view(-1, 3, 8)[-1, 0, -1:].view(torch.bfloat16).float()[0])
                main.wait_stream(side)
            torch.cuda.synchronize()
            ref = torch.arange(1, trials + 1, device=dev, dtype=torch.float32)
            print(f"last main op before the fork = {last:7s}, side reader = {reader:7s}: stale in "
                  f"{int((R != ref).sum())} of {trials}", flush=True)


if __name__ == "__main__":
    main()
