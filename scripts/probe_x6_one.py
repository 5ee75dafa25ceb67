"""Run one x6 GEMM (fc1 forward shape, cfg from argv) 30 times: a target for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat

kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 0
M = 111_000
g = torch.Generator(device="cuda").manual_seed(0)
if kind == "wgrad":
    A = torch.randn(2, M, 512, device="cuda", generator=g)
    B = torch.relu(torch.randn(2, M, 576, device="cuda", generator=g))
    for _ in range(30):
        nat.x6_gemm_tn(A, B, cfg=cfg)
else:
    N, K = (512, 576) if kind == "fwd" else (576, 512)
    A = torch.relu(torch.randn(2, M, K, device="cuda", generator=g))
    Bp = nat.x6_split(torch.randn(2, N, K, device="cuda", generator=g))
    for _ in range(30):
        nat.x6_gemm_nt(A, Bp, cfg=cfg)
torch.cuda.synchronize()
print("done")
