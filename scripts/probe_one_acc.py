"""Probe (round 6): fc1's plane-operand NT GEMMs with ONE accumulator per tile (merlin_h3p.hip k_h3_pq<..., ONE>: the
lo planes brought back to scale in registers, all three products into one fp32 accumulator) against the
two-accumulator kernels, at the update's shapes: the input gradient (N = 576, K = 512: cfg 62 vs 65 / 66) and the
forward's shape (N = 512, K = 576: cfg 60 vs 64 / 67 / 68).  HIP-event time per launch (median of 3 rounds, alternating
in one process) and each kernel's error against float64 in the units of tests/test_gpu_h3.py (max |C - C64| /
sum_k |a_k b_k|), beside torch's fp32 GEMM on the same operands.
The no-DMA ablations (cfg 61 / 64 / 67) exist only in a -DMERLIN_PROBES build (make -C ppo-2dgrid_amd
EXTRA=-DMERLIN_PROBES); results: profiles/r06k_one_acc.log, r06r_order.log.
    python scripts/probe_one_acc.py [U] [reps] [cfgs]"""
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


def err(C, C64, den):
    return float(((C.double() - C64).abs() / den.clamp_min(1e-300)).max())


def main():
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 111000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cfgs = [int(c) for c in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = {
        # input gradient: dz [U, 512] (sparse-ish, ~1e-6) x W^T -> [U, 576]
        "dgrad": (576, 512, [62, 66, 67, 61]),
        # forward's shape: a3 [U, 576] (ReLU output) x W4 [512, 576]^T -> [U, 512]
        "fwd": (512, 576, [60]),
    }
    for name, (N, K, cs) in shapes.items():
        if cfgs:
            cs = [c for c in cs if c in cfgs]
        if name == "dgrad":
            A = torch.randn(2, U, K, device=dev, generator=g) * 1e-6
            A = A * (torch.rand(2, U, K, device=dev, generator=g) > 0.3)
        else:
            A = torch.relu(torch.randn(2, U, K, device=dev, generator=g))
            A = A * torch.exp2(torch.randint(-8, 3, (2, U, 1), device=dev, generator=g).float())
        B = torch.randn(2, N, K, device=dev, generator=g) / K ** 0.5
        amA, amB = nat.h3_amax(A), nat.h3_amax(B)
        Ap, Bp = nat.h3_split(A, amA), nat.h3_split(B, amB)
        flop = 2 * 2 * U * N * K * 3  # executed f16 MFMA work (three plane products per fp32 product)
        outs, times = {}, {c: [] for c in cs}
        for _ in range(3):
            for c in cs:
                outs[c] = torch.empty(2, U, N, device=dev)
                times[c].append(timeit(lambda: nat.h3_gemm_nt_planes(Ap, amA, Bp, amB, cfg=c, out=outs[c]), reps))
        rows = slice(0, min(U, 20000))
        C64 = torch.bmm(A[:, rows].double(), B.double().transpose(1, 2))
        den = torch.bmm(A[:, rows].abs().double(), B.abs().double().transpose(1, 2))
        e32 = err(torch.bmm(A[:, rows], B.transpose(1, 2)), C64, den)
        print(f"{name} (U={U}, N={N}, K={K}): torch fp32 error {e32:.3e}")
        for c in cs:
            t = sorted(times[c])[1]
            print(f"  cfg {c}: {t:7.1f} us per launch, {flop / t / 1e6:6.0f} TF/s executed ({flop / t / 1e6 / 2500:.3f} of "
                  f"the dense f16 peak), error {err(outs[c][:, rows], C64, den):.3e}")
        ref = cs[0]
        for c in cs[1:]:
            d = (outs[c] - outs[ref]).abs().max().item()
            print(f"  cfg {c} vs {ref}: max |diff| {d:.3e}, equal {torch.equal(outs[c], outs[ref])}")


if __name__ == "__main__":
    main()
