"""Probe: the dQ passes of merlin/windows.py _WindowConv3.backward at the bench size.  Builds the
bench rollout's WindowPlan (4096 envs x 256 steps, after `--iters` PPO iterations), takes one
minibatch of 131072 samples and times, with HIP events:
  pass 1  R = per-patch sums of the ReLU-masked dY3 rows (merlin_segment_sum_masked)
  direct  dQ from R, 9 entries per patch (the two-pass form)
  bands   S from R (3 per patch) then dQ from S (3 per band) -- at several item lengths
and prints the sizes that set their traffic (patches, live patches, bands, windows)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from merlin import MerlinVecEnv
    from merlin import _native as nat
    from merlin.dedup import FrameGroups
    from merlin.ppo import PPO
    from merlin.windows import P2_OF, SegmentPlan, WindowPlan

    dev = torch.device("cuda", 0)
    N, T = 4096, 256
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, ent_coef=0.05, device=dev)
    for _ in range(args.iters):
        agent.update(agent.collect_rollouts())
    agent.collect_rollouts()
    codes = agent.buf.flat_codes
    plan = WindowPlan(codes, FrameGroups(codes))
    B = codes.shape[0]
    mb = plan.epoch_minibatches(torch.randperm(B, device=dev), B // 8)[0]
    U = int(mb.groups.numel())
    K = plan.num_patches
    live = plan.kid.index_select(0, mb.groups).reshape(-1)
    kmap = torch.full((K,), -1, dtype=torch.int32, device=dev)
    kmap[live] = live
    nlive = int((kmap >= 0).sum())
    print(f"F={plan.num_frames} U={U} windows={plan.num_windows} patches={K} live={nlive} bands={plan.num_bands}",
          flush=True)
    pairs = torch.unique(plan.kid.index_select(0, mb.groups).long() * 9 + torch.arange(9, device=dev)).numel()
    print(f"minibatch (p3, patch) pairs {pairs} of {U * 9} frame-positions ({U * 9 / pairs:.2f}x)", flush=True)
    if os.environ.get("PAIRS_ONLY"):
        return
    dY3 = torch.randn(2, U * 9, 64, device=dev)
    Y3 = torch.randn(2, U * 9, 64, device=dev)
    rows = plan.num_windows * 9
    R = nat.segment_sum(dY3, plan.patch_plan, K, slot=mb.slot, sub=9, mask=Y3, fill=False)
    for L in (128, 256, 512, 1024):
        pp = SegmentPlan(plan.patch_plan.key, plan.patch_plan.idx, L)
        t = timeit(lambda: nat.segment_sum(dY3, pp, K, slot=mb.slot, sub=9, mask=Y3, fill=False, out=R))
        print(f"pass 1 (patch sums, masked) L={L}: {t:.1f} us", flush=True)
    # direct: (patch, tap) -> window at tap, 9 per patch
    ks, ko = torch.sort(plan.kid.reshape(-1).long(), stable=True)
    first = torch.ones(ks.numel(), dtype=torch.bool, device=dev)
    first[1:] = ks[1:] != ks[:-1]
    e = ko[first]
    p2 = torch.tensor(P2_OF, dtype=torch.int64, device=dev)
    subw = plan.wid[e // 9].long().gather(1, p2[e % 9])
    dk, do = torch.sort((subw * 9 + torch.arange(9, device=dev)).reshape(-1), stable=True)
    out = torch.empty(2, rows, 64, device=dev)
    for L in (256, 1024):
        dplan = SegmentPlan(dk, do // 9, L)
        t = timeit(lambda: nat.segment_sum(R, dplan, rows, slot=kmap, sub=1, out=out))
        print(f"direct dQ from R, L={L}: {t:.1f} us", flush=True)
    ref = out.clone()
    S = torch.empty(2, plan.num_bands, 64, device=dev)
    for LS in (64, 128, 256):
        sp = SegmentPlan(plan.band_plan.key, plan.band_plan.idx, LS)
        ts = timeit(lambda: nat.segment_sum(R, sp, plan.num_bands, slot=kmap, sub=1, out=S))
        for LQ in (16, 32, 64):
            qp = SegmentPlan(plan.dq_plan.key, plan.dq_plan.idx, LQ)
            tq = timeit(lambda: nat.segment_sum(S, qp, rows, out=out))
            print(f"bands: S L={LS} {ts:.1f} us + dQ L={LQ} {tq:.1f} us  max|diff| vs direct "
                  f"{float((out - ref).abs().max()):.3g}", flush=True)
    # compacted live patches (a per-minibatch plan): R rows renumbered densely
    order = torch.nonzero(kmap >= 0).squeeze(1)
    Rc = R[:, order].contiguous()
    newid = torch.full((K,), -1, dtype=torch.int64, device=dev)
    newid[order] = torch.arange(order.numel(), device=dev)
    bk = plan.band_plan.key.long()
    bi = newid[plan.band_plan.idx.long()]
    keep = bi >= 0
    cp = SegmentPlan(bk[keep], bi[keep], 1024)
    print(f"bands from compacted R ({order.numel()} rows): {timeit(lambda: nat.segment_sum(Rc, cp, plan.num_bands, out=S)):.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
