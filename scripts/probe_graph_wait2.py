"""Probe: ordering around a HIP-graph replay that follows a cross-stream join, with no host synchronisation between
trials (as PPO._sgd issues its minibatch steps).  Trial k: the main stream forks a side stream that spins and then
writes X = k; main runs its own kernels, joins the side stream (wait_stream), replays a captured graph G (Y = X),
then plain kernels record Y[0] and X[0] into slot k of two result arrays.  Both must read k: the replay and the
plain kernels after the join, before the next trial's side write.
    python scripts/probe_graph_wait2.py [trials]"""
import sys

import torch


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    n = 1 << 22
    X, Y, Z = (torch.zeros(n, device=dev) for _ in range(3))
    RY = torch.zeros(trials, device=dev)
    RX = torch.zeros(trials, device=dev)
    tick = torch.zeros(1, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        Y.copy_(X)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        Y.copy_(X)
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    for use_graph in (True, False):
        for tickit in (False, True):
            RY.zero_()
            RX.zero_()
            torch.cuda.synchronize()
            for k in range(1, trials + 1):
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(1_500_000)
                    X.fill_(float(k))
                for _ in range(10):
                    Z.mul_(1.0)
                main.wait_stream(side)
                if tickit:
                    tick.add_(0)
                if use_graph:
                    g.replay()
                else:
                    Y.copy_(X)
                RY[k - 1].copy_(Y[-1])
                RX[k - 1].copy_(X[-1])
            torch.cuda.synchronize()
            ref = torch.arange(1, trials + 1, device=dev, dtype=torch.float32)
            print(f"{'graph' if use_graph else 'plain':5s} {'with tick' if tickit else 'no tick':9s}: "
                  f"Y stale in {int((RY != ref).sum())}, X stale in {int((RX != ref).sum())} of {trials}", flush=True)


if __name__ == "__main__":
    main()
