"""Probe: the per-update planning of PPO._sgd at the bench state (merlin.dedup.FrameGroups, merlin.windows.WindowPlan,
WindowPlan.update_minibatches(bulk=True)), wall time with the stream drained around each stage, median of `reps`.
    python scripts/probe_plan.py [warm iterations] [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin.dedup import FrameGroups
from merlin.ppo import PPO
from merlin.windows import WindowPlan


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(4096, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, ent_coef=0.05, device=dev)
    for _ in range(warm):
        agent.update(agent.collect_rollouts())
    agent.collect_rollouts()
    codes = agent.buf.flat_codes
    B = codes.shape[0]
    perms = [torch.randperm(B, device=dev) for _ in range(10)]
    ts = {"FrameGroups": [], "WindowPlan": [], "update_minibatches": [], "update_minibatches(lazy)": []}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fg = FrameGroups(codes)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        plan = WindowPlan(codes, fg)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        plan.update_minibatches(perms, B // 8, bulk=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        plan.update_minibatches(perms, B // 8, bulk=False)
        torch.cuda.synchronize()
        ts["update_minibatches(lazy)"].append((time.perf_counter() - t3) * 1e3)
        ts["FrameGroups"].append((t1 - t0) * 1e3)
        ts["WindowPlan"].append((t2 - t1) * 1e3)
        ts["update_minibatches"].append((t3 - t2) * 1e3)
    print({k: round(statistics.median(v), 2) for k, v in ts.items()}, "ms;", f"frames {plan.num_frames} windows "
          f"{plan.num_windows} patches {plan.num_patches} bands {plan.num_bands}", flush=True)


if __name__ == "__main__":
    main()
