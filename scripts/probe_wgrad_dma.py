"""Standalone timing of fc1's weight gradient at the update's shape (U rows, 32 splits): the register-staged TN on
fp32 operands (cfg 0, k_h3_tng), on dz planes (AQ), on both planes (AQ+BQ), and the LDS-DMA TN on both planes
(cfg 20, k_h3_tq); bit equality of the plane variants."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat

U = int(sys.argv[1]) if len(sys.argv) > 1 else 111111
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
dz = torch.randn(2, U, 512, device=dev, generator=g) * 1e-6
a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
rows = torch.arange(U * 9, dtype=torch.int32, device=dev)
amz, am3 = nat.h3_amax(dz), nat.h3_amax(a3)
dzp, a3p = nat.h3_split(dz, amz), nat.h3_split(a3, am3)
runs = {"tng fp32": lambda: nat.h3_gemm_tn(dz, amz, a3, am3, rows=rows, cfg=0),
        "tng AQ": lambda: nat.h3_gemm_tn(dzp, amz, a3, am3, rows=rows, cfg=0),
        "tng AQ+BQ": lambda: nat.h3_gemm_tn(dzp, amz, a3p, am3, rows=rows, cfg=0),
        "tq (DMA)": lambda: nat.h3_gemm_tn(dzp, amz, a3p, am3, rows=rows, cfg=20)}
outs = {}
for name, fn in runs.items():
    outs[name] = fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    tf = 3 * 2 * 2 * U * 576 * 512 / (us * 1e-6) / 1e12
    print(f"{name:12s} {us:8.1f} us (incl. fold)  executed MFMA {tf:6.1f} TF/s ({tf / 2500:.3f} of 2.5 PF)"
          f"  bits == tng AQ+BQ: {torch.equal(outs[name], outs.get('tng AQ+BQ', outs[name]))}")
