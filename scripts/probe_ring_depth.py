"""Probe (round 6): fc1's plane-operand GEMMs at the update's shape with a deeper LDS-DMA ring.  The DMA of a k step is
latency-bound (DESIGN.md §4 'Round 5': ~31 GB/s per CU at three stages), so the feed should scale with the steps in
flight; k_h3_pq cfg 62 (3 stages, 120 KB) vs cfg 63 (4 stages, 160 KB) on the same planes: HIP-event time per launch,
alternating in one process, and the outputs bit for bit (same products, same order).
    python scripts/probe_ring_depth.py [U] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def timeit(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 111000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    dz = torch.randn(2, U, 512, device=dev, generator=g) * 1e-6
    W = torch.randn(2, 512, 576, device=dev, generator=g) / 24
    Wt = W.transpose(1, 2).contiguous()
    amWt, amz = nat.h3_amax(Wt), nat.h3_amax(dz)
    Htp = nat.h3_split(Wt, amWt)
    pdz = nat.h3_split(dz, amz)
    flop = 2 * 2 * U * 576 * 512 * 3  # executed f16 MFMA work (three plane products per fp32 product)
    outs = {}
    times = {c: [] for c in (62, 63)}
    for _ in range(3):
        for c in (62, 63):
            outs[c] = torch.empty(2, U, 576, device=dev)
            times[c].append(timeit(lambda: nat.h3_gemm_nt_planes(pdz, amz, Htp, amWt, cfg=c, out=outs[c]), reps))
    for c, t in times.items():
        t = sorted(t)[len(t) // 2]
        print(f"dgrad cfg {c}: {t:.1f} us per launch, {flop / t / 1e6:.0f} TF/s executed ({flop / t / 1e6 / 2500:.3f} "
              f"of the dense f16 peak)")
    print("bitwise equal:", torch.equal(outs[62], outs[63]))


if __name__ == "__main__":
    main()
