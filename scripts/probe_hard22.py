"""Probe: bench.py's hard 22x22 tier (BASELINE cfg 4) under switches, rollout and update timed apart.
    python scripts/probe_hard22.py [settings, e.g. base,noheadsepi,noreuse]"""
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin import _native as nat
from merlin import fast_step as FS
from merlin.ppo import PPO


def run(name, dev, N=4096, T=256, warm=2, iters=3):
    nat.H3_HEADS_EPILOGUE = "noheadsepi" not in name
    FS.PATCH_REUSE = False if "noreuse" in name else "gather"
    env = MerlinVecEnv(N, difficulty="hard", size=22, seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=10, batch_size=N * T,
                minibatch_size=N * T // 8, vf_coef=0.5, ent_coef=0.05, device=dev)
    rows = []
    for i in range(warm + iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lv = agent.collect_rollouts()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        agent.update(lv)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if i >= warm:
            rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
    print(f"{name:12s} rollout {[round(r, 1) for r, _ in rows]} ms  update {[round(u, 1) for _, u in rows]} ms  "
          f"distinct {agent.last_distinct_frac:.4f} windows {agent.last_num_windows} "
          f"pack {'Qall' if agent.rollout_all_windows else 'per-frame'}", flush=True)
    env.close()
    del agent
    torch.cuda.empty_cache()


def main():
    dev = torch.device("cuda", 0)
    for name in (sys.argv[1] if len(sys.argv) > 1 else "base,noheadsepi").split(","):
        run(name, dev)


if __name__ == "__main__":
    main()
