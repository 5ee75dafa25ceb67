"""Probe: the fast step's window-GEMM backward alone (merlin/fast_step.py after conv3's dQ: da2w = dQ W3r^T on
hipBLASLt, dW3r = a2w^T dQ as the split-K product + its sum, relu_bwd with the bias gradient) at the update's shape
(nw windows, 2 towers), against merlin_window_gemm_bwd (csrc/merlin_winbwd.hip), HIP events, median of `reps`.
    python scripts/probe_window_bwd.py [nw] [reps]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat
from merlin.actor_critic import _splitk_bmm_tn


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
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 6571
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    a2w = torch.relu(torch.randn(2, nw, 64, device=dev, generator=g))
    W3r = torch.randn(2, 64, 576, device=dev, generator=g) * 0.05
    dQ = torch.randn(2, nw, 576, device=dev, generator=g) * 1e-3
    gW = torch.empty(2, 64, 576, device=dev)
    gb = torch.empty(2, 64, device=dev)

    def dgrad():
        da2w = torch.bmm(dQ, W3r.transpose(1, 2))
        nat.relu_bwd(a2w, da2w, out=da2w, out_bias=gb)

    def wgrad():
        _splitk_bmm_tn(a2w, dQ, max(1, nw // 256), min_chunk=128, name="gemm_window_wgrad", out=gW)

    def both():
        dgrad()
        wgrad()

    def hip():
        nat.window_gemm_bwd(a2w, dQ, W3r, out_db2=gb, out_dW3r=gW)

    print(f"nw {nw}: dgrad + relu_bwd {timed(dgrad, reps):.1f} us  wgrad {timed(wgrad, reps):.1f} us  "
          f"both {timed(both, reps):.1f} us  merlin_window_gemm_bwd {timed(hip, reps):.1f} us", flush=True)


if __name__ == "__main__":
    main()
