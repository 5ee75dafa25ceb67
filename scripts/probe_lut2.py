"""Time the conv2-table kernels at the bench's minibatch size (131072 frames) on env
observation codes (a random-action rollout of the mediumhard envs) and on uniform codes."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
import torch  # noqa: E402

from merlin import MerlinVecEnv, _native as nat  # noqa: E402
from merlin.actor_critic import CNNActorCritic  # noqa: E402

dev = torch.device("cuda:0")
N, T, MB = 4096, 32, 131072
env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
codes = torch.zeros((T + 1, N, 8), dtype=torch.int32, device=dev)
env.reset(out=codes[0])
acts = torch.randint(0, 3, (T, N), device=dev)
for t in range(T):
    env.step_into(acts[t].contiguous(), codes[t + 1], torch.empty(N, device=dev), None, None, torch.empty(N, device=dev))
flat = codes[1:].reshape(-1, 8).contiguous()
uni = torch.randint(0, 5, (MB, 49), device=dev)
ac = CNNActorCritic((56, 56, 3), 3).to(dev)
T2 = ac.conv2_tables().detach().contiguous()


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for name, cd in (("env", flat), ):
    idx = torch.randint(0, cd.shape[0], (MB,), device=dev)
    g = torch.randn(2, 16, MB * 25, 4, device=dev)
    g[g < 0] = 0
    print(name, "fwd ms", timeit(lambda: nat.conv2_lut_fwd(cd, idx, T2)), flush=True)
    cm = cd.index_select(0, idx)
    print(name, "hist ms", timeit(lambda: nat.conv2_lut_bwd(cm, g)), flush=True)
