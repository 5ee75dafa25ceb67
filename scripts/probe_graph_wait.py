"""Probe: is a HIP-graph replay ordered after a cross-stream wait (Stream.wait_stream -> hipStreamWaitEvent) that
is the last thing on the stream before the replay?  The main stream forks a side stream that spins, then writes
X = k; main runs its own kernels meanwhile, waits for the side stream and replays a captured graph that copies X
into Y (graph kinds: one copy kernel; a memset node first; a three-kernel chain).  Y != k afterwards = the replay
ran before the side stream's write.  Each mode is also run with one plain kernel between the wait and the replay.
    python scripts/probe_graph_wait.py [trials]"""
import sys

import torch


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    X = torch.zeros(1 << 20, device=dev)
    Y = torch.zeros_like(X)
    Z = torch.zeros(1 << 22, device=dev)
    tick = torch.zeros(1, device=dev)
    flag = torch.zeros(4, dtype=torch.int32, device=dev)

    def copy():
        Y.copy_(X)

    def memset_first():
        flag.zero_()
        Y.copy_(X)

    def chain():
        flag.add_(1)
        Y.copy_(X)
        Y.mul_(1.0)

    graphs = {}
    for name, fn in (("copy", copy), ("memset_first", memset_first), ("chain", chain)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graphs[name] = g
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    for name, g in graphs.items():
        for tickit in (False, True):
            bad = 0
            for k in range(1, trials + 1):
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(3_000_000)
                    X.fill_(float(k))
                for _ in range(20):  # main-stream work beside the side stream
                    Z.mul_(1.0)
                main.wait_stream(side)
                if tickit:
                    tick.add_(0)
                g.replay()
                torch.cuda.synchronize()
                bad += int(float(Y[0]) != float(k) or float(Y[-1]) != float(k))
            print(f"{name:13s} {'wait+tick+replay' if tickit else 'wait+replay':16s}: {bad} of {trials} replays "
                  f"read X before the side stream wrote it", flush=True)


if __name__ == "__main__":
    main()
