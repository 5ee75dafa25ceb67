"""Probe (round 5): where the plane-operand NT GEMM's time goes -- k_h3_ntg AP (cfg 42, 128 x 256) against its
ablations: 47 no DMA in the main loop, 48 no MFMAs, 49 the DMA stream alone.  HIP-event time per launch.
(The ablation configs are compiled only with -DMERLIN_PROBES: make -C ppo-2dgrid_amd EXTRA=-DMERLIN_PROBES.)
    python scripts/probe_h3_ablate.py [U] [reps] [cfgs...]"""
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
    cfgs = [int(c) for c in sys.argv[3:]] or [42, 47, 48, 49]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
    W = torch.randn(2, 512, 576, device=dev, generator=g) / 24
    b = torch.zeros(2, 512, device=dev)
    amW, am3 = nat.h3_amax(W), nat.h3_amax(a3)
    Hp = nat.h3_split(W, amW)
    pa3 = nat.h3_split(a3, am3).view(torch.float32)
    out = torch.empty(2, U, 512, device=dev)
    flop = 3 * 2 * 2 * U * 576 * 512
    res = {c: [] for c in cfgs}
    for _ in range(3):
        for c in cfgs:
            res[c].append(timeit(lambda c=c: nat.h3_gemm_nt(pa3, am3, Hp, amW, bias=b, cfg=c, out=out), reps))
    for c in cfgs:
        us = min(res[c])
        print(f"cfg {c:3d} {us:8.1f} us  executed MFMA-equivalent {flop / us / 1e6:7.1f} TF/s "
              f"({flop / us / 1e6 / 2500:.3f} of 2.5 PF); bytes staged {2 * U * (576 * 4) * 2 / us / 1e3:.0f} GB/s A "
              f"x2 tiles", flush=True)


if __name__ == "__main__":
    main()
