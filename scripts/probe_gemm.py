"""GEMM shapes of conv2/conv3 as im2col GEMMs (both towers), fp32 (not part of the product)."""
import time
import torch

dev = torch.device("cuda:0")


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def t_ms(fn, reps=5):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


B = 131072
for name, M, K, N in (("conv2", B * 25, 512, 64), ("conv3", B * 9, 576, 64), ("fc1", B, 576, 512)):
    A = torch.rand(2, M, K, device=dev)
    W = torch.rand(2, K, N, device=dev)
    dZ = torch.rand(2, M, N, device=dev)
    fl = 2 * 2 * M * K * N
    f = t_ms(lambda: torch.bmm(A, W))
    w = t_ms(lambda: torch.bmm(A.transpose(1, 2), dZ))
    d = t_ms(lambda: torch.bmm(dZ, W.transpose(1, 2)))
    f1 = t_ms(lambda: A[0] @ W[0])
    log(f"{name} M={M} K={K} N={N}: fwd bmm {f:.2f} ms {fl / f / 1e9:.1f} TF | wgrad {w:.2f} ms {fl / w / 1e9:.1f} TF"
        f" | dgrad {d:.2f} ms {fl / d / 1e9:.1f} TF | single fwd {f1:.2f} ms {fl / 2 / f1 / 1e9:.1f} TF")
    del A, W, dZ
    torch.cuda.empty_cache()
log("done")
