"""Probe the three-plane bf16 GEMMs (csrc/merlin_gemm.hip) at fc1's update shapes: exactness of
the plane split, error against float64 beside torch's fp32 GEMM (hipBLASLt), and time per tile
configuration.  Run on the GPU box: python scripts/probe_x6.py [M]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def rel_err(C, C64, den):
    return float(((C.double() - C64).abs() / den.clamp_min(1e-300)).max())


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 111_000
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    # split exactness over many magnitudes
    x = torch.randn(1 << 20, device=dev, generator=g) * torch.exp2(torch.randint(-60, 60, (1 << 20,), device=dev,
                                                                                   generator=g).float())
    x[:8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0e38, 1e-30, 1.0000001, -7.25], device=dev)
    P = nat.x6_split(x.view(-1, 64))
    back = nat.x6_join(P).view(-1)
    print("split exact:", bool(torch.equal(back, x)), "mismatches", int((back != x).sum()))

    for name, (N, K, cfgs) in {"fwd": (512, 576, [0]), "dgrad": (576, 512, [1])}.items():
        # fc1-like operands: A >= 0 sparse-ish activations, B weights
        A = torch.relu(torch.randn(2, M, K, device=dev, generator=g))
        B = torch.randn(2, N, K, device=dev, generator=g) / K ** 0.5
        bias = torch.randn(2, N, device=dev, generator=g) * 0.1
        Ap, Bp = A, nat.x6_split(B)
        rows = slice(0, min(M, 20000))
        C64 = torch.bmm(A[:, rows].double(), B.double().transpose(1, 2))
        den = torch.bmm(A[:, rows].abs().double(), B.abs().double().transpose(1, 2))
        Cref = torch.bmm(A, B.transpose(1, 2))
        e_ref = rel_err(Cref[:, rows], C64, den)
        t_ref = timeit(lambda: torch.bmm(A, B.transpose(1, 2)))
        flops = 2 * 2 * M * N * K
        print(f"[{name}] M={M} N={N} K={K}: torch fp32 bmm {t_ref:.1f} us ({flops / t_ref / 1e6:.1f} TF), "
              f"max err/sum|ab| {e_ref:.3e}")
        for cfg in cfgs:
            try:
                C = nat.x6_gemm_nt(Ap, Bp, cfg=cfg)
            except nat.MerlinNativeError as ex:
                print(f"  cfg {cfg}: {ex}")
                continue
            e = rel_err(C[:, rows], C64, den)
            tail = float((C[:, -7:] - Cref[:, -7:]).abs().max())
            t = timeit(lambda: nat.x6_gemm_nt(Ap, Bp, cfg=cfg))
            Cb = nat.x6_gemm_nt(Ap, Bp, bias=bias, cfg=cfg)
            eb = float((Cb - torch.relu(C + bias.unsqueeze(1))).abs().max())
            print(f"  cfg {cfg}: {t:.1f} us ({flops / t / 1e6:.1f} TF-fp32-equiv), max err/sum|ab| {e:.3e}, "
                  f"tail rows {tail:.2e}, bias+relu epilogue diff {eb:.2e}")

    # weight gradient: out[t] = dz^T a3 (Kd = M rows, 512 x 576)
    Mj, Nc = 512, 576
    dz = torch.randn(2, M, Mj, device=dev, generator=g) * (torch.rand(2, M, Mj, device=dev, generator=g) > 0.5)
    a3 = torch.relu(torch.randn(2, M, Nc, device=dev, generator=g))
    dzp, a3p = dz, a3
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    den = torch.bmm(dz.abs().double().transpose(1, 2), a3.abs().double())
    Wref = torch.bmm(dz.transpose(1, 2), a3)
    flops = 2 * 2 * M * Mj * Nc
    t_ref = timeit(lambda: torch.bmm(dz.transpose(1, 2), a3))
    print(f"[wgrad] Kd={M}: torch fp32 bmm {t_ref:.1f} us ({flops / t_ref / 1e6:.1f} TF), "
          f"max err/sum|ab| {rel_err(Wref, W64, den):.3e}")
    for cfg in (3,):
        for splits in (16, 32):
            try:
                W = nat.x6_gemm_tn(dzp, a3p, splits=splits, cfg=cfg)
            except nat.MerlinNativeError as ex:
                print(f"  cfg {cfg}: {ex}")
                break
            e = rel_err(W, W64, den)
            t = timeit(lambda: nat.x6_gemm_tn(dzp, a3p, splits=splits, cfg=cfg))
            print(f"  cfg {cfg} splits {splits}: {t:.1f} us ({flops / t / 1e6:.1f} TF-fp32-equiv), "
                  f"max err/sum|ab| {e:.3e}")


if __name__ == "__main__":
    main()
