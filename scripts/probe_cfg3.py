"""Device memory and time of one PPO iteration at a given (envs, k_steps, minibatches, epochs) shape, one process.

    python scripts/probe_cfg3.py N T MB EPOCHS

Used to size tests/test_gpu_dp.py's cfg-3 case (8 ranks x 4096 envs on one device, against one process over the
32,768 concatenated envs): prints torch.cuda.max_memory_allocated() after the rollout and after the update."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin.ppo import PPO


def main():
    N, T, MB, EP = (int(a) for a in sys.argv[1:5])
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(5)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // MB, update_epochs=EP, ent_coef=0.05, device=dev)
    for it in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lv = agent.collect_rollouts()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        m_roll = torch.cuda.max_memory_allocated()
        stats = agent.update(lv)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"shape N={N} T={T} MB={MB} epochs={EP} iter {it}: rollout {1e3 * (t1 - t0):.0f} ms, update "
              f"{1e3 * (t2 - t1):.0f} ms, max allocated after rollout {m_roll / 2**30:.2f} GiB, after update "
              f"{torch.cuda.max_memory_allocated() / 2**30:.2f} GiB, reserved {torch.cuda.memory_reserved() / 2**30:.2f}"
              f" GiB, fast {agent._wstep is not None}, windows {agent.last_num_windows}, distinct/sample "
              f"{agent.last_distinct_frac:.3f}, stats {stats}", flush=True)


if __name__ == "__main__":
    main()
