"""Probe (round 6): the plane-operand NT GEMMs' time split into main loop, DMA and epilogue, at the update's shapes
(input gradient N = 576, K = 512: cfg 62; forward N = 512, K = 576: cfg 60), against the probe-build ablations of
merlin_h3p.hip k_h3_pq (wrong results on purpose): ABL 1 no DMA in the k loop (67 / 74), ABL 2 no tile stores (70 /
72), ABL 3 neither (71 / 73).  One block of 144 KB LDS holds a CU, so a tile's prologue (two k steps' DMA) and
epilogue (its C stores) do not overlap another tile's MFMAs.  HIP-event time per launch, median of 3 alternating
rounds.  Run with the probe library: make -C ppo-2dgrid_amd -B EXTRA=-DMERLIN_PROBES LIB=lib/libmerlin_hip_probe.so,
MERLIN_HIP_LIB=ppo-2dgrid_amd/lib/libmerlin_hip_probe.so python scripts/probe_epilogue.py [U] [reps]"""
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
    # (round 6, profiles/r06ag_epilogue.log: 4-wave blocks on a 2-stage ring, two blocks per CU so that one block's
    # epilogue runs beside the other's MFMAs -- 128 x 128, 256 x 64, 64 x 256 -- took 434 / 468-483 / 464 us, slower
    # than one 8-wave block per CU; those configs were removed again)
    shapes = {"dgrad": (576, 512, {62: "full", 70: "no stores", 67: "no DMA", 71: "neither"}),
              "fwd": (512, 576, {60: "full", 72: "no stores", 74: "no DMA", 73: "neither"})}
    for name, (N, K, cs) in shapes.items():
        A = torch.relu(torch.randn(2, U, K, device=dev, generator=g))
        B = torch.randn(2, N, K, device=dev, generator=g) / K ** 0.5
        amA, amB = nat.h3_amax(A), nat.h3_amax(B)
        Ap, Bp = nat.h3_split(A, amA), nat.h3_split(B, amB)
        out = torch.empty(2, U, N, device=dev)
        flop = 2 * 2 * U * N * K * 3
        times = {c: [] for c in cs}
        for _ in range(3):
            for c in cs:
                times[c].append(timeit(lambda c=c: nat.h3_gemm_nt_planes(Ap, amA, Bp, amB, cfg=c, out=out), reps))
        print(f"{name} (U={U}, N={N}, K={K}); C = {2 * U * N * 4 / 1e6:.0f} MB written by the full kernel")
        for c, what in cs.items():
            t = sorted(times[c])[1]
            print(f"  cfg {c} ({what:9s}): {t:7.1f} us, {flop / t / 1e6 / 2500:.3f} of the dense f16 peak", flush=True)


if __name__ == "__main__":
    main()
