"""Where a FOMAML meta step (BASELINE cfg 5: 32 tasks x 256 support + 256 query) spends its time:
support rollout, support loss + inner grads, query rollout, query loss + grads, meta Adam.
python scripts/probe_fomaml.py [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import numpy as np
import torch

from merlin import ScenarioCreator
from merlin import fomaml as F


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    fm = F.FOMAML(ScenarioCreator(), lr_inner=0.01, lr_outer=3e-4, device=dev, difficulty="mediumhard")
    acc = {}

    def timed(name, fn):
        def w(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            acc.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
            return r
        return w

    fm.collect_trajectory = timed("rollout", fm.collect_trajectory)
    fm.compute_loss = timed("loss_fwd", fm.compute_loss)
    grad0 = torch.autograd.grad
    torch.autograd.grad = timed("autograd", grad0)
    rs = np.random.RandomState(42)
    for it in range(iters):
        acc.clear() if it == 1 else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fm.meta_train_step(rs.choice(100000, 32, replace=False), k_support=256, k_query=256)
        torch.cuda.synchronize()
        print(f"iter {it}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    for k, v in acc.items():
        print(f"{k:10s} calls {len(v)} total {sum(v):.1f} ms  each {[round(x, 1) for x in v]}")


if __name__ == "__main__":
    main()
