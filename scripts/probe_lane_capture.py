"""Probe (round 6): capturing multi-stream rollouts as one HIP graph -- a pure-torch fork / join pattern shaped like a
rollout stepped as K env-range lanes (main -> K lane streams; mode a: each lane also forks a refill stream per step and
joins it before its next step, which segfaults in hipStreamEndCapture on ROCm 7 / torch 2.10; mode a1: the refills in
the lane, which captures).  The lane rollout itself (merlin_env_act_step_range, in-lane refills) measured slower than
one chain and was not kept: profiles/r06o_rollout.log, DESIGN.md section 4 'Round 6'.
    python scripts/probe_lane_capture.py a|a1 [K]"""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch


def pattern(K, T=16, side=True):
    dev = torch.device("cuda", 0)
    x = torch.zeros(K, 1024, device=dev)
    ls = [torch.cuda.Stream() for _ in range(K)]
    rs = [torch.cuda.Stream() for _ in range(K)]

    def body():
        main = torch.cuda.current_stream()  # the capturing stream inside torch.cuda.graph
        for j in range(K):
            ls[j].wait_stream(main)
        pend = [False] * K
        for t in range(T):
            for j in range(K):
                with torch.cuda.stream(ls[j]):
                    y = x[j] * 2 + 1
                    if pend[j]:
                        ls[j].wait_stream(rs[j])
                    x[j].copy_(y)
                if side:
                    rs[j].wait_stream(ls[j])
                    with torch.cuda.stream(rs[j]):
                        x[j].add_(0.5)
                    pend[j] = True
                else:
                    with torch.cuda.stream(ls[j]):
                        x[j].add_(0.5)
        for j in range(K):
            ls[j].wait_stream(rs[j])
            main.wait_stream(ls[j])

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g.replay()
    torch.cuda.synchronize()
    print("pattern ok", K, flush=True)


if __name__ == "__main__":
    mode = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    pattern(K, side=mode == "a")
