"""Probe: the weight stage's table kernels alone (csrc/merlin_stage.hip: k_stage_fwd, k_stage_bwd_h + k_stage_bwd_w),
HIP events, median of `reps` launches, random weights of the update's shapes.
    python scripts/probe_stage.py [reps]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat
from merlin.actor_critic import CNNActorCritic


def timed(f, reps):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    ac = CNNActorCritic((56, 56, 3), 3).to(dev)
    atlas, idx, koff, kv = ac.stage_consts(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    W1 = torch.randn(2, 32, 3, 8, 8, device=dev, generator=g) * 0.05
    b1 = torch.randn(2, 32, device=dev, generator=g) * 0.05
    W2 = torch.randn(2, 64, 32, 4, 4, device=dev, generator=g) * 0.05
    HT, T2 = nat.stage_tables_fwd(W1, b1, W2, atlas, idx)
    dT2 = torch.randn_like(T2)
    fwd = timed(lambda: nat.stage_tables_fwd(W1, b1, W2, atlas, idx, HT=HT, T2=T2), reps)
    bwd = timed(lambda: nat.stage_tables_bwd(W2, HT, dT2, atlas, koff, kv), reps)
    print(f"stage fwd {fwd:.1f} us   stage bwd (h + w) {bwd:.1f} us   T2 sum {float(T2.double().sum()):.10e}",
          flush=True)


if __name__ == "__main__":
    main()
