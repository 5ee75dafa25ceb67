"""Probe: does PyTorch TunableOp (exhaustive hipBLASLt / rocBLAS solution search per GEMM shape)
find faster kernels than the default heuristic for the update's fc1 GEMMs at the bench shape?
Times fwd (bias+ReLU epilogue), dgrad and the split-K wgrad chunk GEMM before and after tuning."""
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
    from merlin.actor_critic import _splitk_bmm_tn, bias_relu_bmm

    dev = torch.device("cuda", 0)
    U, K, H = int(os.environ.get("U", 115712)), 576, 512
    a3 = torch.randn(2, U, K, device=dev)
    W = torch.randn(2, H, K, device=dev) * 0.05
    b = torch.randn(2, H, device=dev)
    dz = torch.randn(2, U, H, device=dev)
    fl = 2 * 2 * U * K * H
    cases = {
        "fwd": lambda: bias_relu_bmm(a3, W.transpose(1, 2), b),
        "fwd_bmm+k_bias_relu": lambda: nat.bias_relu_(torch.bmm(a3, W.transpose(1, 2)), b),
        "fwd_2mm+k_bias_relu": lambda: nat.bias_relu_(torch.stack([a3[t] @ W[t].t() for t in range(2)]), b),
        "dgrad": lambda: torch.bmm(dz, W),
        "wgrad": lambda: _splitk_bmm_tn(a3, dz, 32),
    }
    base = {k: timeit(f) for k, f in cases.items()}
    ref = {k: f() for k, f in cases.items()}
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(int(os.environ.get("TUNE_MS", 200)))
    torch.cuda.tunable.set_filename(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "tunable.csv"))
    for k, f in cases.items():
        f()  # tunes
    torch.cuda.synchronize()
    for k, f in cases.items():
        t = timeit(f)
        d = float((f() - ref[k]).abs().max())
        print(f"{k}: default {base[k]:.0f} us ({fl / base[k] / 1e6:.0f} TF)  tuned {t:.0f} us "
              f"({fl / t / 1e6:.0f} TF)  max|diff| {d:.3g}", flush=True)


if __name__ == "__main__":
    main()
