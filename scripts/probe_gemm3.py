"""Probe: the update's fc1 GEMMs at the bench shape (both towers, U distinct frames x 576 -> 512)
under each BLAS backend torch offers on ROCm (hipBLASLt / rocBLAS), and fc1 forward with the bias +
ReLU fused into the GEMM epilogue (torch._addmm_activation) against bmm + merlin's k_bias_relu."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from merlin import _native as nat

    dev = torch.device("cuda", 0)
    U, K, H = 115738, 576, 512
    a3 = torch.randn(2, U, K, device=dev)
    W = torch.randn(2, H, K, device=dev) * 0.05
    b = torch.randn(2, H, device=dev)
    dz = torch.randn(2, U, H, device=dev)
    fl = 2 * 2 * U * K * H
    for backend in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(backend)
        except Exception as e:  # noqa: BLE001
            print(backend, "unavailable:", e)
            continue
        t_f = timeit(lambda: torch.bmm(a3, W.transpose(1, 2)))
        t_d = timeit(lambda: torch.bmm(dz, W))
        t_w = timeit(lambda: torch.bmm(a3.transpose(1, 2), dz))
        print(f"{backend}: fwd {t_f:.0f} us ({fl / t_f / 1e6:.0f} TF)  dgrad {t_d:.0f} us ({fl / t_d / 1e6:.0f} TF)  "
              f"wgrad(plain) {t_w:.0f} us ({fl / t_w / 1e6:.0f} TF)", flush=True)
        t_br = timeit(lambda: nat.bias_relu_(torch.bmm(a3, W.transpose(1, 2)), b))
        z = torch.empty(2, U, H, device=dev)

        def fused():
            for t in range(2):
                torch._addmm_activation(b[t], a3[t], W[t].t(), out=z[t])
        try:
            t_fu = timeit(fused)
            ref = nat.bias_relu_(torch.bmm(a3, W.transpose(1, 2)), b)
            fused()
            d = float((z - ref).abs().max())
            print(f"  bmm + k_bias_relu {t_br:.0f} us   2x _addmm_activation {t_fu:.0f} us  max|diff| {d:.3g}", flush=True)
        except Exception as e:  # noqa: BLE001
            print("  _addmm_activation failed:", e)
        t_mm = timeit(lambda: [torch.mm(a3[t], W[t].t()) for t in range(2)])
        print(f"  2x mm (fwd) {t_mm:.0f} us", flush=True)


if __name__ == "__main__":
    main()
