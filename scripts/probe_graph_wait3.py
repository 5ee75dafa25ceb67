"""Probe: cross-stream ordering with the library's own launches (hipLaunchKernelGGL on torch's stream handle,
merlin._native) at the edges of a fork / join, no host synchronisation between trials.  Trial k: main forks a side
stream that runs a long library kernel (h3 TN GEMM) and then the library's x6_split of a tensor filled with k into P;
main runs its own kernels, joins (wait_stream), then reads P with the first op after the join being (a) a library
kernel (x6_join), (b) a torch kernel, (c) a graph replay of x6_join; the value read goes to slot k.
    python scripts/probe_graph_wait3.py [trials]"""
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
    J = torch.zeros(1 << 16, device=dev)
    Z = torch.zeros(1 << 22, device=dev)
    R = torch.zeros(trials, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        J.copy_(nat.x6_join(P))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        J.copy_(nat.x6_join(P))
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    for mode in ("library", "torch", "graph"):
        R.zero_()
        torch.cuda.synchronize()
        for k in range(1, trials + 1):
            side.wait_stream(main)
            with torch.cuda.stream(side):
                nat.h3_gemm_tn(dz, amz, a3, am3, out=W)
                nat.x6_split(vals[k], out=P)
            for _ in range(10):
                Z.mul_(1.0)
            main.wait_stream(side)
            if mode == "library":
                J.copy_(nat.x6_join(P))
            elif mode == "torch":
                J.copy_(P.view(-1, 3, 8)[:, 0].contiguous().view(torch.bfloat16).float().view(-1))
            else:
                g.replay()
            R[k - 1].copy_(J[-1])
        torch.cuda.synchronize()
        ref = torch.arange(1, trials + 1, device=dev, dtype=torch.float32)
        print(f"first op after the join = {mode:7s}: stale in {int((R != ref).sum())} of {trials}", flush=True)


if __name__ == "__main__":
    main()
