"""Per-component timing probe (prints as it goes).  Not part of the product."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch
from merlin import MerlinVecEnv, _native as nat
from merlin.actor_critic import CNNActorCritic

def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)

bench = int(os.environ.get("PROBE_BENCH", "0"))
torch.backends.cudnn.benchmark = bool(bench)
dev = torch.device("cuda:0")
log("device", torch.cuda.get_device_name(0), "cudnn.benchmark", bench)

def timeit(fn, reps=5):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps

N = 4096
env = MerlinVecEnv(N, seed=777, device=dev)
codes = env.reset().clone()
acts = torch.randint(0, 3, (N,), device=dev)
log("env step (1 launch, N=4096) ms", timeit(lambda: env.step_into(acts, env.obs), 50))
big = torch.randint(0, 2**31 - 1, (131072, 8), device=dev, dtype=torch.int32) & 0x33333333
out = torch.empty((131072, 3, 56, 56), device=dev)
ms = timeit(lambda: nat.expand_obs(big, out=out, scale=1/255))
log("expand 131072 nchw ms", ms, "GB/s", 131072 * 37632 / ms / 1e6)
torch.manual_seed(0)
ac = CNNActorCritic((56, 56, 3), 3).to(dev)
FWD = 4_970_496 * 2
for B in (4096,):
    x = torch.rand((B, 3, 56, 56), device=dev)
    with torch.no_grad():
        log("compiling fwd", B)
        ms = timeit(lambda: ac.act(x, prescaled=True))
    log(f"act fwd B={B} ms {ms:.3f}  TFLOP/s {B * FWD / ms / 1e9:.1f}")
opt = torch.optim.Adam(ac.parameters(), lr=3e-4)
import threading
def hb():
    while True:
        time.sleep(50); log("heartbeat")
threading.Thread(target=hb, daemon=True).start()
for B in [int(b) for b in os.environ.get("PROBE_BATCHES", "8192,32768,131072").split(",")]:
    x = torch.rand((B, 3, 56, 56), device=dev)
    a = torch.randint(0, 3, (B,), device=dev)
    def step():
        lp, ent, v = ac.evaluate(x, a, prescaled=True)
        loss = -lp.mean() + v.pow(2).mean() - 0.05 * ent.mean()
        opt.zero_grad(set_to_none=True); loss.backward()
        torch.nn.utils.clip_grad_norm_(ac.parameters(), 0.5); opt.step()
    log("compiling fwd+bwd", B)
    ms = timeit(step, 3)
    log(f"fwd+bwd+adam B={B} ms {ms:.2f}  TFLOP/s {B * 25.67e6 / ms / 1e9:.1f}")
log("done")
