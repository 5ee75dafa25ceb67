"""Find the host<->device synchronisations inside one PPO update (and one rollout) of the bench
workload: torch.cuda.set_sync_debug_mode("warn") with every warning's Python call site counted."""
import collections
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))

sites = collections.Counter()


def show(message, category, filename, lineno, file=None, line=None):
    st = [f for f in traceback.extract_stack()[:-1] if "merlin" in f.filename or "bench" in f.filename]
    key = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:][::-1])
    sites[key] += 1


def main():
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    dev = torch.device("cuda", 0)
    N, T = 4096, 256
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, ent_coef=0.05, device=dev)
    for _ in range(3):
        agent.update(agent.collect_rollouts())
    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    lv = agent.collect_rollouts()
    agent.update(lv)
    torch.cuda.set_sync_debug_mode("default")
    print(f"{sum(sites.values())} synchronising calls in one rollout + update", flush=True)
    import time

    from merlin.dedup import FrameGroups
    from merlin.windows import WindowPlan
    codes = agent.buf.flat_codes
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fg = FrameGroups(codes)
        t1 = time.perf_counter()
        plan = WindowPlan(codes, fg)
        t2 = time.perf_counter()
        perms = [torch.randperm(codes.shape[0], device=dev) for _ in range(10)]
        plan.update_minibatches(perms, codes.shape[0] // 8)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"FrameGroups {1e3 * (t1 - t0):.1f} ms, WindowPlan {1e3 * (t2 - t1):.1f} ms, "
              f"update_minibatches {1e3 * (t3 - t2):.1f} ms (wall, per update)", flush=True)
    for k, c in sites.most_common(40):
        print(f"{c:5d}  {k}", flush=True)


if __name__ == "__main__":
    main()
