"""How many distinct observations does a bench rollout hold?  (4096 mediumhard envs x 256
random-action steps; distinct 32-byte code rows overall and inside random 131072-frame
minibatches.)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
import torch  # noqa: E402

from merlin import MerlinVecEnv  # noqa: E402

dev = torch.device("cuda:0")
for diff, size in (("mediumhard", 16), ("hard", 22)):
    N, T, MB = 4096, 256, 131072
    env = MerlinVecEnv(N, diff, size=size, seed=777, device=dev)
    codes = torch.zeros((T + 1, N, 8), dtype=torch.int32, device=dev)
    env.reset(out=codes[0])
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for t in range(T):
        a = torch.randint(0, 3, (N,), device=dev, generator=g)
        env.step_into(a, codes[t + 1], torch.empty(N, device=dev), None, None, torch.empty(N, device=dev))
    flat = codes[:T].reshape(-1, 8)
    u = torch.unique(flat, dim=0)
    print(diff, "rollout frames", flat.shape[0], "distinct", u.shape[0], f"{u.shape[0] / flat.shape[0]:.3f}")
    perm = torch.randperm(flat.shape[0], device=dev)
    for k in range(3):
        mb = flat[perm[k * MB:(k + 1) * MB]]
        um = torch.unique(mb, dim=0)
        print("  minibatch", k, "distinct", um.shape[0], f"{um.shape[0] / MB:.3f}")
