"""Host queueing time vs GPU time of PPO.update at the bench configuration: is the host ahead of the GPU?
python scripts/probe_host.py [warmup_iters]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin import _native as nat
from merlin.ppo import PPO


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda")
    env = MerlinVecEnv(4096, difficulty="mediumhard", size=16, seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, lr=3e-4, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, update_epochs=10, ent_coef=0.05,
                device=dev)
    for _ in range(warm):
        agent.update(agent.collect_rollouts())
    torch.cuda.synchronize()
    for timers in (False, True, False):
        if timers:
            nat.KernelTimer.start()
        lv = agent.collect_rollouts()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        agent.update(lv)
        e1.record()
        t_ret = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) * 1e3
        if timers:
            nat.KernelTimer.stop()
        mb = agent.last_host_mb_ms
        print(f"timers={timers}: gpu update {e0.elapsed_time(e1):.1f} ms, host loop {agent.last_host_loop_ms:.1f} ms, "
              f"update() returned after {t_ret:.1f} ms, wall {t_all:.1f} ms; host per minibatch: first {mb[0]:.2f}, "
              f"median {statistics.median(mb[1:]):.2f}, max {max(mb[1:]):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
