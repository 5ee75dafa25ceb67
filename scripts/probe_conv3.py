"""Probe: k_window_conv3 alone at the bench state (one minibatch of the bench rollout's WindowPlan, random Q),
HIP events, median of `reps`, plus checksums of Y3 and the ReLU bit words so two library builds (MERLIN_HIP_LIB)
can be compared for identical output.  python scripts/probe_conv3.py [warm iterations] [reps]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin import _native as nat
from merlin.dedup import FrameGroups
from merlin.ppo import PPO
from merlin.windows import WindowPlan


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(4096, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, ent_coef=0.05, device=dev)
    for _ in range(warm):
        agent.update(agent.collect_rollouts())
    agent.collect_rollouts()
    codes = agent.buf.flat_codes
    plan = WindowPlan(codes, FrameGroups(codes))
    B = codes.shape[0]
    g = torch.Generator(device=dev).manual_seed(5)
    mb = plan.update_minibatches([torch.randperm(B, device=dev, generator=g)], B // 8, bulk=True)[0][0]
    nw = plan.num_windows
    Q = torch.randn(2, nw, 576, device=dev, generator=g)
    b3 = torch.randn(2, 64, device=dev, generator=g)
    am = torch.zeros(2, dtype=torch.int32, device=dev)
    variants = {"all rows": lambda: nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am),
                "patch reuse": lambda: nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am, rep_row=mb.rep_row),
                "reps only + masks": lambda: nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am,
                                                              rep_row=mb.rep_row, copy=2),
                "reps only": lambda: nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am, rep_row=mb.rep_row,
                                                      copy=0)}
    outs = {}
    for name, f in variants.items():
        am.zero_()
        Y3, bits = f()
        outs[name] = (Y3, bits, am.clone())
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        print(f"{name}: lib {os.path.basename(nat.LIB_PATH)} U={int(mb.groups.numel())} windows={nw} "
              f"reps={int((mb.rep_row == torch.arange(mb.rep_row.numel(), device=dev, dtype=torch.int32)).sum())}: {statistics.median(ts):.1f} us  "
              f"Y3 sum {float(Y3.double().sum()):.10e}  "
              f"bits xor {int(bits.view(-1).cpu().numpy().astype('uint64').sum(dtype='uint64'))}", flush=True)
    (a, ab, aa), (b, bb, ba) = list(outs.values())[:2]
    print("identical:", torch.equal(a, b), torch.equal(ab, bb), torch.equal(aa, ba), flush=True)


if __name__ == "__main__":
    main()
