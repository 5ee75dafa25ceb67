"""A/B of the x6 NT GEMM variants (csrc/merlin_gemm.hip cfgs) at fc1's update shapes, one process,
interleaved rounds, median per cfg; each variant checked bitwise against the base kernel (same
per-element operation order).  python scripts/probe_x6_il.py [U] [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def ev_time(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 116192
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    cfgs = [int(c) for c in os.environ.get("CFGS", "").split(",") if c] or None
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = {"fwd": (512, 576, True, [0, 20, 21, 24, 25, 2, 10, 30, 26, 28]),
              "dgrad": (576, 512, False, [1, 22, 23, 13, 32, 27])}
    if os.environ.get("PROF"):
        shapes = {"fwd": (512, 576, True, [0, 20]), "dgrad": (576, 512, False, [1, 22])}
    for name, (N, K, use_bias, cl) in shapes.items():
        cl = [c for c in cl if cfgs is None or c in cfgs or c in (0, 1)]
        A = torch.relu(torch.randn(2, U, K, device=dev, generator=g)) if use_bias else \
            torch.randn(2, U, K, device=dev, generator=g) * (torch.rand(2, U, K, device=dev, generator=g) > 0.5)
        Bp = nat.x6_split(torch.randn(2, N, K, device=dev, generator=g) / K ** 0.5)
        if os.environ.get("ZEROS"):  # operand data toggling no bits: the matrix cores' power draw drops
            A.zero_()
            Bp.zero_()
        bias = torch.randn(2, N, device=dev, generator=g) * 0.1 if use_bias else None
        Ap = nat.x6_split(A)  # A as planes for the cfg >= 30 kernels
        AA = lambda c, X=None: (nat.x6_split(X) if X is not None else Ap) if c >= 30 else (A if X is None else X)  # noqa: E731
        ref = nat.x6_gemm_nt(A, Bp, bias=bias, cfg=cl[0])
        # error vs float64 on the first rows, relative to sum |a b| (no bias: the raw product)
        Bf = nat.x6_join(Bp).view(2, N, K)
        rows = slice(0, 8192)
        C64 = torch.bmm(A[:, rows].double(), Bf.double().transpose(1, 2))
        den = torch.bmm(A[:, rows].abs().double(), Bf.abs().double().transpose(1, 2))
        e_ref = float(((torch.bmm(A[:, rows], Bf.transpose(1, 2)).double() - C64).abs() / den).max())
        print(f"[{name}] hipBLASLt fp32 max err/sum|ab| {e_ref:.3e}")
        ok = {}
        for c in cl:
            try:
                out = nat.x6_gemm_nt(AA(c), Bp, bias=bias, cfg=c)
                raw = nat.x6_gemm_nt(AA(c, A[:, rows].contiguous()), Bp, cfg=c)
                err = float(((raw.double() - C64).abs() / den).max())
                ok[c] = (bool(torch.equal(out, ref)), err)
            except nat.MerlinNativeError as ex:
                print(name, c, ex)
        times = {c: [] for c in ok}
        for _ in range(rounds):
            for c in ok:
                times[c].append(ev_time(lambda: nat.x6_gemm_nt(AA(c), Bp, bias=bias, cfg=c)))
        ex = 6 * 2 * 2 * U * N * K
        for c in ok:
            med = statistics.median(times[c])
            print(f"[{name}] cfg {c:2d}: median {med:8.1f} us  min {min(times[c]):8.1f}  "
                  f"{ex / med / 1e6:7.1f} TF executed ({ex / med / 1e6 / 2500:.3f} of 2.5 PF)  bitwise-equal {ok[c][0]} err {ok[c][1]:.3e}",
                  flush=True)


if __name__ == "__main__":
    main()
