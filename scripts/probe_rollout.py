"""In-process A/B of rollout settings at the bench workload (4096 envs x 256 steps, captured rollout graph):
one agent, each setting's graph captured once, then rollouts timed alternately.
    python scripts/probe_rollout.py [rounds] [settings, e.g. 1,2,4 (refill_every) or x6,h3r12,h3r2,h3r12_qbmm]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin.ppo import PPO


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    vals = (sys.argv[2] if len(sys.argv) > 2 else "1,2").split(",")
    from merlin import _native as nat
    from merlin import actor_critic as AC

    def setting(v):
        from merlin import ppo as PPO_MOD

        PPO_MOD.ROLLOUT_STEP_FALLBACK = v.endswith("fb")  # e.g. 1fb: the per-step fallback pass launched anyway
        if v.rstrip("fb").isdigit():
            agent.refill_every = int(v.rstrip("fb"))
            return
        AC.ROLLOUT_FC1_H3 = v.startswith("h3")
        nat.H3_NT_CFG["rollout"] = next((int(t[3:]) for t in v.split("_") if t[:3] == "h3r"), 12)
        AC.QALL_H3 = "qbmm" not in v
        from merlin import ppo as PPO_MOD

        PPO_MOD.ROLLOUT_SCALE_ROWS = "zero" not in v  # e.g. h3r12_zero: the per-step zeroing launch
        nat.H3_HEADS_EPILOGUE = "noheadsepi" not in v  # e.g. h3r12_noheadsepi: fc1's z + merlin_act_heads
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(4096, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, ent_coef=0.05, device=dev)
    for _ in range(int(os.environ.get("WARM", "6"))):  # the bench's state: episode lengths change with training
        agent.update(agent.collect_rollouts())
    graphs = {}
    for v in vals:
        setting(v)
        agent._graph = None
        agent.collect_rollouts()  # eager + capture
        graphs[v] = agent._graph
    times = {v: [] for v in vals}
    for _ in range(rounds):
        for v in vals:
            agent._graph = graphs[v]
            setting(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            agent.collect_rollouts()
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) * 1e3)
    for v in vals:
        print(f"{v}: median {statistics.median(times[v]):.2f} ms per rollout  all "
              f"{[round(x, 2) for x in times[v]]}", flush=True)


if __name__ == "__main__":
    main()
