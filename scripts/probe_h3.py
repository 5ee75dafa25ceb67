"""Probe: fc1's three GEMMs at the update's shape (U distinct frames per minibatch, both towers), the exact
three-plane bf16 form (merlin_x6_*, six products) against the two-plane f16 form (merlin_h3_*, three products),
alternating in one process; HIP-event time per launch and the executed MFMA rate.
    python scripts/probe_h3.py [U] [reps] [h3 nt cfg fwd] [h3 nt cfg dgrad] [h3 tn cfg]"""
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
    cf, cd, ct = (int(sys.argv[i]) if len(sys.argv) > i else d for i, d in ((3, 0), (4, 1), (5, 0)))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
    dz = torch.randn(2, U, 512, device=dev, generator=g) * 1e-6
    W = torch.randn(2, 512, 576, device=dev, generator=g) / 24
    Wt = W.transpose(1, 2).contiguous()
    b = torch.zeros(2, 512, device=dev)
    Wp, Wtp = nat.x6_split(W), nat.x6_split(Wt)
    amW, amWt = nat.h3_amax(W), nat.h3_amax(Wt)
    Hp, Htp = nat.h3_split(W, amW), nat.h3_split(Wt, amWt)
    am3 = nat.h3_amax(a3)
    amz = nat.h3_amax(dz)
    flop = 2 * 2 * U * 576 * 512
    pa3, pdz = nat.h3_split(a3, am3), nat.h3_split(dz, amz)
    runs = {
        "x6 fwd": (lambda: nat.x6_gemm_nt(a3, Wp, bias=b, cfg=nat.X6_NT_CFG["fwd"]), 6),
        "h3 fwd": (lambda: nat.h3_gemm_nt(a3, am3, Hp, amW, bias=b, cfg=cf), 3),
        "x6 dgrad": (lambda: nat.x6_gemm_nt(dz, Wtp, cfg=nat.X6_NT_CFG["dgrad"]), 6),
        "h3 dgrad": (lambda: nat.h3_gemm_nt(dz, amz, Htp, amWt, cfg=cd), 3),
        "x6 wgrad": (lambda: nat.x6_gemm_tn(dz, a3), 6),
        "h3 wgrad": (lambda: nat.h3_gemm_tn(dz, amz, a3, am3, cfg=ct), 3),
        "h3 wgrad pl": (lambda: nat.h3_gemm_tn(pdz, amz, pa3, am3, cfg=ct), 3),
        "h3 amax a3": (lambda: nat.h3_amax(a3, out=am3), 0),
    }
    if cf < 20:  # the DMA-staged kernels have no plane output
        runs["h3 fwd +pl"] = (lambda: nat.h3_gemm_nt(a3, am3, Hp, amW, bias=b, cfg=cf, planes_out=pa3), 3)
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, (fn, prods) in runs.items():
            res[k].append(timeit(fn, reps))
    for k, (fn, prods) in runs.items():
        us = min(res[k])
        line = f"{k:12s} {us:8.1f} us"
        if prods:
            line += f"  fp32-equiv {flop / us / 1e6:7.1f} TF/s  executed MFMA {prods * flop / us / 1e6:7.1f} TF/s " \
                    f"({prods * flop / us / 1e6 / 2500:.3f} of 2.5 PF)"
        print(line, flush=True)
    # accuracy at this shape against float64 (one tower, first 4096 rows)
    n = 4096
    C64 = a3[0, :n].double() @ W[0].double().T
    den = a3[0, :n].abs().double() @ W[0].abs().double().T
    for k, C in (("x6", nat.x6_gemm_nt(a3, Wp, cfg=nat.X6_NT_CFG["fwd"])), ("h3", nat.h3_gemm_nt(a3, am3, Hp, amW, cfg=cf)),
                 ("f32", torch.bmm(a3, W.transpose(1, 2)))):
        print(f"fwd err/sum|ab| {k}: {float(((C[0, :n].double() - C64).abs() / den).max()):.3e}")


if __name__ == "__main__":
    main()
