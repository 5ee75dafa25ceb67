"""Probe: is a plain launch after a HIP-graph replay ordered after the WHOLE graph?  The graph (captured once): some
long elementwise kernels, then merlin_h3_amax of a small tensor S (a memset node zeroing the result, then an atomicMax
kernel) -- the fast step's forward-graph tail.  Trial k (no host synchronisation between trials): S = k (plain fill),
replay, then a plain copy records the graph's amax result into slot k.  Slot k must hold k.
    python scripts/probe_graph_then.py [trials]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    Z = torch.zeros(1 << 24, device=dev)
    S = torch.zeros(2, 64, device=dev)
    am = torch.zeros(2, dtype=torch.int32, device=dev)
    R = torch.zeros(trials, dtype=torch.int32, device=dev)
    R2 = torch.zeros(trials, dtype=torch.int32, device=dev)

    def body(nk):
        for _ in range(nk):
            Z.mul_(1.0)
        nat.h3_amax(S, out=am)

    for nk in (0, 8):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body(nk)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body(nk)
        for reader in ("torch", "library"):
            R.zero_()
            torch.cuda.synchronize()
            for k in range(1, trials + 1):
                S.fill_(float(k))
                g.replay()
                if reader == "torch":
                    R[k - 1].copy_(am[1])
                else:  # a library kernel reading am right after the replay: h3_split of S with scale am
                    P = nat.h3_split(S, am)
                    R[k - 1].copy_(P.view(torch.float16)[1, 0].float().to(torch.int32))  # hi plane of S[1][0]
            torch.cuda.synchronize()
            if reader == "torch":
                ref = torch.tensor([torch.tensor(float(k)).view(torch.int32).item() for k in range(1, trials + 1)],
                                   dtype=torch.int32, device=dev)
            else:  # S[1][0] = k scaled into [2^14, 2^15): 2^(14 - floor(log2 k)) * k
                import math
                ref = torch.tensor([int(k * 2 ** (14 - math.floor(math.log2(k)))) for k in range(1, trials + 1)],
                                   dtype=torch.int32, device=dev)
            print(f"graph with {nk} leading kernels, reader {reader:7s}: wrong in {int((R != ref).sum())} of {trials}"
                  f"; got {R[:4].tolist()} want {ref[:4].tolist()}", flush=True)
    # the same body eagerly
    S.fill_(3.0)
    body(0)
    torch.cuda.synchronize()
    print("eager: am =", am.tolist(), "=", am.view(torch.float32).tolist())
    S.fill_(5.0)
    g.replay()
    torch.cuda.synchronize()
    print("one replay, synchronised: am =", am.tolist(), "=", am.view(torch.float32).tolist())


if __name__ == "__main__":
    main()
