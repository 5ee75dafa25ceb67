"""Probe: resets per step in the 2M-env tier (bench.py env_large_tier) and the step / auto-reset
split, timed with HIP events around each launch (single-step launches, random actions)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def main():
    from merlin import MerlinVecEnv

    dev = torch.device("cuda", 0)
    for n in (1 << 21, 4096):
        env = MerlinVecEnv(n, difficulty="mediumhard", size=16, seed=31337, device=dev)
        env.reset()
        g = torch.Generator(device=dev)
        g.manual_seed(9)
        T = 32
        used = torch.zeros(n, dtype=torch.bool, device=dev)  # slot consumed since the last refill
        acts = torch.randint(0, 3, (T, n), device=dev, generator=g)
        obs = torch.empty((T, n, 8), dtype=torch.int32, device=dev)
        rew = torch.empty((T, n), dtype=torch.float32, device=dev)
        done = torch.empty((T, n), dtype=torch.float32, device=dev)
        for t in range(T):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            env.step_into(acts[t], obs[t], rew[t], None, None, done[t])
            e1.record()
            torch.cuda.synchronize()
            d = done[t] > 0
            fb = int((d & used).sum())
            used |= d
            if (t + 1) % 16 == 0:
                used.zero_()
            print(f"n={n} step {t}: resets {int(d.sum())} ({float(done[t].mean()) * 100:.3f} %) "
                  f"empty-slot resets {fb} step+autoreset {e0.elapsed_time(e1) * 1e3:.1f} us", flush=True)
        env.errors()
        env.close()


if __name__ == "__main__":
    main()
