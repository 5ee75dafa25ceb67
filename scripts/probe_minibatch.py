"""Time the pieces of one PPO minibatch step of the bench (after a real rollout): dedup
grouping, table build, tower forward, heads+loss, backward, clip+Adam.  Each segment is
bracketed by a synchronize so the numbers do not overlap (diagnostic only)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
import torch  # noqa: E402

from merlin import MerlinVecEnv  # noqa: E402
from merlin.dedup import FrameGroups  # noqa: E402
from merlin.ppo import PPO  # noqa: E402

dev = torch.device("cuda:0")
N, T = 4096, 256
env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
torch.manual_seed(777)
agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, ent_coef=0.05, device=dev)
lv = agent.collect_rollouts()
buf = agent.buf
B = N * T
adv, ret = agent._advantages(buf.rewards, buf.values, buf.dones, lv, buf.adv, buf.returns)
codes = buf.flat_codes
acts, lpo, adv, ret = buf.actions.reshape(B), buf.logprobs.reshape(B), adv.reshape(B), ret.reshape(B)
ac = agent.ac
seg = {}


def tick(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    seg[name] = seg.get(name, 0.0) + (t - t0) * 1e3
    return t


torch.cuda.synchronize()
FrameGroups(codes)
t = time.perf_counter()
fg = FrameGroups(codes)
t = tick("frame_groups (once per update)", t)
reps = 8
for r in range(reps + 2):
    if r == 2:
        seg = {k: v for k, v in seg.items() if 'once' in k}
    mb = torch.randperm(B, device=dev)[: B // 8]
    t = tick("randperm", t)
    g = fg.minibatch(mb)
    t = tick("minibatch groups", t)
    T2 = ac.conv2_tables()
    t = tick("conv2_tables fwd", t)
    logits, value = ac._forward_codes_lut2(codes, g[0]) if False else (None, None)
    from merlin.actor_critic import _Conv2LutTower
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    A3 = _Conv2LutTower.apply(T2, torch.stack([ea[2].bias, ec[2].bias]), codes, g[0])
    t = tick("lut tower (lut fwd + im2col3)", t)
    logits, value = ac._tower_tail(A3, g[0].numel())
    t = tick("conv3/fc1/heads fwd", t)
    logits, value = logits.index_select(0, g[1]), value.index_select(0, g[1])
    from merlin.actor_critic import _categorical, _entropy
    logp_all, probs = _categorical(logits)
    lp = logp_all.gather(-1, acts[mb].unsqueeze(-1)).squeeze(-1)
    ent = _entropy(logp_all, probs)
    ratio = torch.exp(lp - lpo[mb])
    a_mb = adv[mb]
    s1 = ratio * a_mb
    s2 = torch.clamp(ratio, 0.8, 1.2) * a_mb
    loss = -torch.min(s1, s2).mean() + 0.5 * ((value - ret[mb]) ** 2).mean() - 0.05 * ent.mean()
    t = tick("gather + loss fwd", t)
    agent.optimizer.zero_grad()
    loss.backward()
    t = tick("backward (all)", t)
    gn = torch.nn.utils.clip_grad_norm_(agent._params, 0.5)
    agent.optimizer.step()
    t = tick("clip + adam", t)
print(f"distinct {g[0].numel()} of {mb.numel()}")
for k, v in seg.items():
    print(f"{k:40s} {v / (1 if 'once' in k else reps):8.3f} ms")

# kernel-level view of one backward
from torch.profiler import ProfilerActivity, profile  # noqa: E402

mb = torch.randperm(B, device=dev)[: B // 8]
g = fg.minibatch(mb)
lp, ent, v = ac.evaluate_codes(codes, acts[mb], index=mb, groups=g)
ratio = torch.exp(lp - lpo[mb])
loss = -torch.min(ratio * adv[mb], torch.clamp(ratio, 0.8, 1.2) * adv[mb]).mean() + 0.5 * ((v - ret[mb]) ** 2).mean() - 0.05 * ent.mean()
agent.optimizer.zero_grad()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CUDA]) as prof:
    loss.backward()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=30, max_name_column_width=70))
