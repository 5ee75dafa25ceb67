"""Rollout fc1 (x6 NT, 4,096 rows x 576 -> 512, both towers) per tile configuration: median of interleaved rounds.
python scripts/probe_rollout_fc1.py [rows]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    a3 = torch.relu(torch.randn(2, n, 576, device=dev, generator=g))
    Wp = nat.x6_split(torch.randn(2, 512, 576, device=dev, generator=g) / 24)
    ref = nat.x6_gemm_nt(a3, Wp, cfg=2)
    cfgs = [int(c) for c in os.environ.get("CFGS", "2,0,20,25,28,29").split(",")]
    times = {c: [] for c in cfgs}
    for c in cfgs:
        err = float((nat.x6_gemm_nt(a3, Wp, cfg=c) - ref).abs().max())
        print(f"cfg {c}: max |diff| vs cfg 2 {err:.3g}", flush=True)
    for _ in range(7):
        for c in cfgs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                nat.x6_gemm_nt(a3, Wp, cfg=c)
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / 20 * 1e3)
    for c in cfgs:
        print(f"cfg {c:2d}: median {statistics.median(times[c]):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
