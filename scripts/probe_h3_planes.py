"""Probe (round 5): fc1's NT GEMMs at the update's shape with BOTH operands already in plane form (k_h3_ntg AP: no
split in the kernel, both operands staged by LDS-DMA) against the current kernels that split the fp32 A operand while
staging (k_h3_ntp cfg 13 / 11); HIP-event time per launch, alternating in one process, bit equality of the outputs.
    python scripts/probe_h3_planes.py [U] [reps]"""
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
    a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
    dz = torch.randn(2, U, 512, device=dev, generator=g) * 1e-6
    W = torch.randn(2, 512, 576, device=dev, generator=g) / 24
    Wt = W.transpose(1, 2).contiguous()
    b = torch.zeros(2, 512, device=dev)
    amW, amWt = nat.h3_amax(W), nat.h3_amax(Wt)
    Hp, Htp = nat.h3_split(W, amW), nat.h3_split(Wt, amWt)
    am3, amz = nat.h3_amax(a3), nat.h3_amax(dz)
    pa3 = nat.h3_split(a3, am3).view(torch.float32)  # [2, U, 576] plane images passed where A goes
    pdz = nat.h3_split(dz, amz).view(torch.float32)
    flop = 2 * 2 * U * 576 * 512
    runs = {"fwd ntp13": (lambda: nat.h3_gemm_nt(a3, am3, Hp, amW, bias=b, cfg=13), "fwd")}
    for c in (50, 51, 60, 61):
        if 512 % {41: 192, 42: 256, 50: 256, 60: 256}.get(c, 128) == 0:
            runs[f"fwd planes{c}"] = ((lambda c=c: nat.h3_gemm_nt(pa3, am3, Hp, amW, bias=b, cfg=c)), "fwd")
    runs["dgrad ntp11"] = (lambda: nat.h3_gemm_nt(dz, amz, Htp, amWt, cfg=11), "dgrad")
    for c in (52, 62):
        runs[f"dgrad planes{c}"] = ((lambda c=c: nat.h3_gemm_nt(pdz, amz, Htp, amWt, cfg=c)), "dgrad")
    runs["split a3"] = (lambda: nat.h3_split(a3, am3), None)
    runs["split dz"] = (lambda: nat.h3_split(dz, amz), None)
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, (fn, _) in runs.items():
            res[k].append(timeit(fn, reps))
    ref = {"fwd": nat.h3_gemm_nt(a3, am3, Hp, amW, bias=b, cfg=13), "dgrad": nat.h3_gemm_nt(dz, amz, Htp, amWt, cfg=11)}
    for k, (fn, kind) in runs.items():
        us = min(res[k])
        line = f"{k:16s} {us:8.1f} us"
        if kind:
            same = torch.equal(fn(), ref[kind])
            line += f"  executed MFMA {3 * flop / us / 1e6:7.1f} TF/s ({3 * flop / us / 1e6 / 2500:.3f} of 2.5 PF)" \
                    f"  bits equal {same}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
