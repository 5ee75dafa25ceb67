"""Diagnostic (round 6): does the fast step's weight stage see parameters loaded after the agent was built?"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
import numpy as np
import torch


def main():
    from merlin import MerlinVecEnv
    from merlin.fast_step import WindowStep
    from merlin.ppo import PPO

    dev = torch.device("cuda", 0)
    g = np.load(os.path.join(REPO, "tests", "golden", "update_grad_ref.npz"))
    env = MerlinVecEnv(1, "mediumhard", seed=1, device=dev)
    torch.manual_seed(0)
    agent = PPO(env, batch_size=8192, minibatch_size=2048, update_epochs=1, device=dev)
    named = list(agent.ac.named_parameters())
    with torch.no_grad():
        for i, (_, p) in enumerate(named):
            p.copy_(torch.from_numpy(g[f"p0_{i}"]).to(dev))
    ws = WindowStep(agent)
    T2s, b2s, W3r, b3, W4p, b4 = ws.stage.forward()
    with torch.no_grad():
        T2t = agent.ac.conv2_tables()
    torch.cuda.synchronize()
    print("stage T2 vs conv2_tables(current params): max |diff|", (T2s - T2t).abs().max().item(), "max |T2|",
          T2t.abs().max().item())
    ea = agent.ac.actor_extractor.network
    print("stage b3[actor] vs param:", (b3[0] - ea[4].bias).abs().max().item(), " W4p row0 vs actor.0.weight:",
          (W4p[0].view(512, 9, 64).transpose(1, 2).reshape(512, 576) - agent.ac.actor[0].weight).abs().max().item())
    # the same after perturbing the actor's conv1 weight in place
    with torch.no_grad():
        ea[0].weight.mul_(1.001)
        T2t2 = agent.ac.conv2_tables()
    T2s2 = ws.stage.forward()[0]
    torch.cuda.synchronize()
    print("after scaling conv1 by 1.001: stage T2 moved", (T2s2 - T2s).abs().max().item(), "torch T2 moved",
          (T2t2 - T2t).abs().max().item(), "stage vs torch", (T2s2 - T2t2).abs().max().item())


if __name__ == "__main__":
    main()
