"""In-process A/B of update-path switches at the bench workload (4096 envs x 256 steps, 10 x 8
minibatches): one agent, warmed up, then the settings alternate iteration by iteration (ABAB...),
so device-to-device and clock differences between gpurun boxes do not enter the comparison.

    python scripts/ab_update.py [iters_per_setting]

Prints ms per iteration (rollout + update) for each setting."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin import windows as W
from merlin.ppo import PPO


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(4096, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, ent_coef=0.05, device=dev)
    for _ in range(3):
        agent.update(agent.collect_rollouts())

    def setter(name):
        def s():
            W.OVERLAP_WGRAD = name != "no_overlap"
            agent.ac.fc1_impl = "hipblaslt" if name == "hipblaslt" else "x6"
        return s

    settings = {n: setter(n) for n in ("x6_overlap", "no_overlap", "hipblaslt")}
    times = {n: [] for n in settings}
    for _ in range(iters):
        for n, s in settings.items():
            s()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            agent.update(agent.collect_rollouts())
            torch.cuda.synchronize()
            times[n].append((time.perf_counter() - t0) * 1e3)
    for n, t in times.items():
        t = sorted(t)
        print(f"{n:12s} median {t[len(t) // 2]:.1f} ms/iter  min {t[0]:.1f}  all {[round(x, 1) for x in times[n]]}")
    print("distinct frames per sample", agent.last_distinct_frac)


if __name__ == "__main__":
    main()
