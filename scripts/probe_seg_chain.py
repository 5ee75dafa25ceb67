"""Probe: conv3's backward chain (merlin/fast_step.py _conv3_backward_bulk: R, S with band marks, dQ, each a
segmented sum + its fix-ups) alone at the bench state, HIP events, median of `reps`; MERLIN_HIP_LIB selects the
library build, so two builds compare on one box.  python scripts/probe_seg_chain.py [warm iterations] [reps]"""
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


def ev(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


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
    U = int(mb.groups.numel())
    dY3 = torch.randn(2, U * 9, 64, device=dev, generator=g)
    bits = torch.randint(-2 ** 62, 2 ** 62, (2, U * 9), device=dev, dtype=torch.int64, generator=g)
    R = torch.empty(2, plan.num_patches, 64, device=dev)
    S = torch.empty(2, plan.num_bands, 64, device=dev)
    dQ = torch.empty(2, plan.num_windows * 9, 64, device=dev)
    bslot = torch.full((plan.num_bands,), -1, dtype=torch.int32, device=dev)
    fR = lambda: nat.segment_sum(dY3, plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9, mask=bits,  # noqa: E731
                                 fill=False, out=R, name="k_seg_sum_R")
    fS = lambda: nat.segment_sum(R, plan.band_plan, plan.num_bands, slot=mb.kmap, sub=1, fill=False,  # noqa: E731
                                 mark=bslot.fill_(-1), out=S, name="k_seg_sum_S")
    fQ = lambda: nat.segment_sum(S, plan.dq_plan, plan.num_windows * 9, slot=bslot, sub=1, out=dQ,  # noqa: E731
                                 name="k_seg_sum_dQ")
    fR(), fS(), fQ()
    print(f"lib {os.path.basename(nat.LIB_PATH)}  U={U} patches={plan.num_patches} bands={plan.num_bands} "
          f"fix rows R/S/dQ {plan.patch_plan.fix.shape[0]}/{plan.band_plan.fix.shape[0]}/{plan.dq_plan.fix.shape[0]}",
          flush=True)
    for fused in (True, False):  # fix-ups inside the launch (merlin_segment_sum_fused) / a k_seg_fix launch
        nat.SEG_FUSED = fused
        fR(), fS(), fQ()
        ts = [ev(f, reps) for f in (fR, fS, fQ)]
        print(f"  {'in-launch fix-ups' if fused else 'k_seg_fix launches'}: R {ts[0]:.1f}  S {ts[1]:.1f}  "
              f"dQ {ts[2]:.1f}  sum {sum(ts):.1f} us", flush=True)
    for name, p in (("R", plan.patch_plan), ("S", plan.band_plan), ("dQ", plan.dq_plan)):
        fx = p.fix[p.fix[:, 0] >= 0]
        span = (fx[:, 2] - fx[:, 1]).float()
        print(f"  {name} fix rows: {fx.shape[0]} live, items spanned max {int(span.max()) if span.numel() else 0}, "
              f"> 64: {int((span > 64).sum())}", flush=True)


if __name__ == "__main__":
    main()
