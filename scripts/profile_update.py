"""Profile: where one minibatch step of the window-path update spends GPU time outside the big
kernels.  Runs the bench's workload for --iters PPO iterations, then records one update's first
`--steps` optimizer steps with torch.profiler and prints GPU kernels grouped by name (total us
per optimizer step) and the CPU ops that launched the most kernels."""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile

    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    dev = torch.device("cuda", 0)
    N, T = 4096, 256
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, ent_coef=0.05, device=dev)
    for _ in range(args.iters):
        agent.update(agent.collect_rollouts())
    agent.collect_rollouts()
    # profile one whole update (update_epochs x 8 optimizer steps)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as p:
        agent.update()
        torch.cuda.synchronize()
    steps = 8 * agent.update_epochs
    agg = collections.defaultdict(lambda: [0, 0.0])
    for e in p.events():
        if e.device_type == torch.autograd.DeviceType.CUDA:
            a = agg[e.name[:90]]
            a[0] += 1
            a[1] += e.device_time
    tot = sum(v[1] for v in agg.values())
    print(f"GPU kernel time per optimizer step: {tot / steps:.0f} us", flush=True)
    for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{t / steps:9.1f} us  {c / steps:6.1f}x  {name}", flush=True)
    print(p.key_averages(group_by_input_shape=False).table(sort_by="self_cpu_time_total", row_limit=25), flush=True)
    # the torch ops behind the glue kernels, with their input shapes and GPU time per step
    rows = []
    for ka in p.key_averages(group_by_input_shape=True):
        if ka.key.startswith("aten::") and ka.self_device_time_total > 0:
            rows.append((ka.self_device_time_total / steps, ka.count / steps, ka.key, str(ka.input_shapes)[:110]))
    for t, c, k, sh in sorted(rows, reverse=True)[:40]:
        print(f"{t:8.1f} us {c:5.1f}x {k:28s} {sh}", flush=True)
    print("-- small ops by shape --", flush=True)
    small = [r for r in rows if r[2] in ("aten::copy_", "aten::cat", "aten::add", "aten::fill_", "aten::mul",
                                         "aten::_index_put_impl_", "aten::zero_", "aten::where", "aten::add_",
                                         "aten::mul_", "aten::sub", "aten::threshold_backward", "aten::relu",
                                         "aten::clone", "aten::index", "aten::gt", "aten::sum")]
    for t, c, k, sh in sorted(small, reverse=True)[:40]:
        print(f"{t:8.1f} us {c:5.1f}x {k:28s} {sh}", flush=True)
    print("-- by op --", flush=True)
    byop = [(ka.self_device_time_total / steps, ka.count / steps, ka.key) for ka in p.key_averages()
            if ka.self_device_time_total > 0]
    for t, c, k in sorted(byop, reverse=True)[:45]:
        print(f"{t:8.1f} us {c:6.1f}x {k}", flush=True)


if __name__ == "__main__":
    main()
