"""Layer-level timing of one CNN tower at the update minibatch (not part of the product).
Prints per layer forward / backward ms and TFLOP/s for NCHW and channels_last, plus a
fused actor+critic conv1 (64 output channels) and grouped conv2/conv3."""
import os
import sys
import time

import torch
import torch.nn.functional as F

B = int(os.environ.get("PB", "131072"))
dev = torch.device("cuda:0")


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def t_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


LAYERS = [  # name, cin, cout, k, s, hin
    ("conv1", 3, 32, 8, 4, 56),
    ("conv2", 32, 64, 4, 2, 13),
    ("conv3", 64, 64, 3, 1, 5),
]


def bench_conv(name, cin, cout, k, s, hin, fmt, groups=1, need_dx=True):
    hout = (hin - k) // s + 1
    x = torch.rand((B, cin * groups, hin, hin), device=dev)
    w = torch.randn((cout * groups, cin, k, k), device=dev) * 0.05
    if fmt == "cl":
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(need_dx)
    w.requires_grad_(True)
    macs = B * groups * cout * hout * hout * cin * k * k
    fwd = t_ms(lambda: F.conv2d(x, w, stride=s, groups=groups))
    y = F.conv2d(x, w, stride=s, groups=groups)
    g = torch.ones_like(y)
    bwd = t_ms(lambda: torch.autograd.grad(y, [x, w] if need_dx else [w], g, retain_graph=True))
    nb = 2 if need_dx else 1
    log(f"{name:8s} {fmt:4s} g{groups} fwd {fwd:7.2f} ms {macs * 2 / fwd / 1e9:6.1f} TF | bwd {bwd:7.2f} ms "
        f"{nb * macs * 2 / bwd / 1e9:6.1f} TF")


def main():
    os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
    log("B", B, "find mode", os.environ.get("MIOPEN_FIND_MODE"))
    for fmt in ("nchw", "cl"):
        for name, cin, cout, k, s, hin in LAYERS:
            bench_conv(name, cin, cout, k, s, hin, fmt, need_dx=(name != "conv1"))
    # tower fusion: conv1 of both towers as one 64-channel conv; conv2/3 as groups=2
    for fmt in ("nchw", "cl"):
        bench_conv("conv1x2", 3, 64, 8, 4, 56, fmt, need_dx=False)
        bench_conv("conv2g2", 32, 64, 4, 2, 13, fmt, groups=2)
        bench_conv("conv3g2", 64, 64, 3, 1, 5, fmt, groups=2)
    a = torch.rand((B, 576), device=dev, requires_grad=True)
    w = torch.randn((512, 576), device=dev, requires_grad=True)
    f = t_ms(lambda: a @ w.t())
    y = a @ w.t()
    g = torch.ones_like(y)
    b = t_ms(lambda: torch.autograd.grad(y, [a, w], g, retain_graph=True))
    m = B * 576 * 512
    log(f"fc1 fwd {f:.2f} ms {2 * m / f / 1e9:.1f} TF | bwd {b:.2f} ms {4 * m / b / 1e9:.1f} TF")
    wb = torch.randn((2, 576, 512), device=dev, requires_grad=True)
    ab = torch.rand((2, B, 576), device=dev, requires_grad=True)
    f = t_ms(lambda: torch.bmm(ab, wb))
    log(f"fc1 x2 bmm fwd {f:.2f} ms {4 * m / f / 1e9:.1f} TF")
    log("done")


if __name__ == "__main__":
    main()
