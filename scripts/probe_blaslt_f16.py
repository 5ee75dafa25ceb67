"""Probe: hipBLASLt's f16-in / f32-out GEMMs (torch.bmm(..., out_dtype=torch.float32)) at fc1's shapes, as the
plane products of the h3 form would use them: hi = A_h B_h^T (K = 576) and lo = [A_h | A_l] [B_l | B_h]^T (K = 1152),
against the hand-written h3 kernel (merlin_h3_gemm_nt) on the same operands.   python scripts/probe_blaslt_f16.py [U]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def timeit(fn, reps=20):
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
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, K, name) in ((512, 576, "fwd"), (576, 512, "dgrad")):
        A = torch.relu(torch.randn(2, U, K, device=dev, generator=g))
        B = torch.randn(2, N, K, device=dev, generator=g) / 24
        Ah, Bh = A.half(), B.half()
        A2 = torch.cat([Ah, Ah], 2)  # [A_h | A_l] stand-in: same shape / cost
        B2t = torch.cat([Bh, Bh], 2).transpose(1, 2)
        Bht = Bh.transpose(1, 2)
        out = torch.empty(2, U, N, device=dev)
        t_hi = timeit(lambda: torch.bmm(Ah, Bht, out_dtype=torch.float32))
        t_lo = timeit(lambda: torch.bmm(A2, B2t, out_dtype=torch.float32))
        # hi accumulated onto lo in one call, if baddbmm takes out_dtype
        try:
            lo = torch.bmm(A2, B2t, out_dtype=torch.float32)
            t_acc = timeit(lambda: torch.baddbmm(lo, Ah, Bht, beta=1.0, alpha=1.0, out_dtype=torch.float32))
        except Exception as e:  # noqa: BLE001
            t_acc = float("nan")
            print("baddbmm out_dtype:", str(e).splitlines()[0][:120])
        amA, amB = nat.h3_amax(A), nat.h3_amax(B)
        Bp = nat.h3_split(B, amB)
        t_h3 = timeit(lambda: nat.h3_gemm_nt(A, amA, Bp, amB, cfg=nat.H3_NT_CFG[name]))
        t_split = timeit(lambda: nat.h3_split(A, amA))
        fl = 2 * 2 * U * N * K
        print(f"{name}: hipBLASLt f16 hi {t_hi:7.1f} us ({fl / t_hi / 1e6:6.0f} TF/s)  lo(K2) {t_lo:7.1f} us "
              f"({2 * fl / t_lo / 1e6:6.0f} TF/s)  baddbmm hi onto lo {t_acc:7.1f}  |  h3 kernel {t_h3:7.1f} us  "
              f"A split {t_split:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
