"""Debug: one bench-size update with fc1 on the h3 GEMMs (fast step and autograd path) -- are the parameters and
update statistics finite, and how far from the x6 update on the same rollout.
    python scripts/debug_h3.py [num_envs] [k_steps]"""
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin.ppo import PPO


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    B = N * T
    agent = PPO(env, batch_size=B, minibatch_size=B // 8, update_epochs=1, ent_coef=0.05, device=dev)
    lv = agent.collect_rollouts()
    sd0 = copy.deepcopy(agent.ac.state_dict())
    opt0 = copy.deepcopy(agent.optimizer.state_dict())
    perm = torch.randperm(B, device=dev)
    agent.perm_fn = lambda n, e: perm
    res = {}
    for impl, fast in (("x6", True), ("h3", True), ("h3", False)):
        agent.ac.load_state_dict(sd0)
        agent.optimizer.load_state_dict(opt0)
        agent.ac.fc1_impl = impl
        agent.fast_step = fast
        stats = agent.update(lv)
        torch.cuda.synchronize()
        ps = [p.detach().clone() for p in agent.ac.parameters()]
        bad = [k for (k, _), p in zip(agent.ac.named_parameters(), ps) if not torch.isfinite(p).all()]
        print(impl, "fast" if fast else "autograd", {k: round(v, 6) for k, v in stats.items()}, "non-finite:", bad,
              flush=True)
        if agent._wstep is not None and fast:
            print("  amax act", agent._wstep.amax_act.view(torch.float32).tolist(), "amaxW",
                  agent._wstep.stage.amaxW.view(torch.float32).tolist(), flush=True)
        res[(impl, fast)] = ps
    for key in (("h3", True), ("h3", False)):
        d = max(float((a - b).abs().max()) for a, b in zip(res[("x6", True)], res[key]))
        print("max |param diff| x6 vs", key, d)


if __name__ == "__main__":
    main()
