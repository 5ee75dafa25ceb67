"""Probe: where k_seg_sum_dQ's time goes at the bench size.  Builds the bench rollout's WindowPlan
(4096 envs x 256 steps, random-init policy, after `--iters` PPO iterations), takes one minibatch of
131072 samples and times merlin_segment_sum on (a) the rollout-level list with the minibatch slot
map (what the update runs) and (b) the same minibatch's entries pre-compacted (no slot map)."""
import argparse
import os
import sys
import time

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
    from merlin.windows import SegmentPlan, WindowPlan

    dev = torch.device("cuda", 0)
    N, T = 4096, 256
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, ent_coef=0.05, device=dev)
    for _ in range(args.iters):
        agent.update(agent.collect_rollouts())
    agent.collect_rollouts()
    codes = agent.buf.flat_codes
    fg = FrameGroups(codes)
    plan = WindowPlan(codes, fg)
    B = codes.shape[0]
    idxs = torch.randperm(B, device=dev)
    mb = plan.epoch_minibatches(idxs, B // 8)[0]
    U = int(mb.groups.numel())
    part = plan.conv3_blocks[0]
    print(f"F={plan.num_frames} U={U} windows={plan.num_windows} list={part.nnz} valid~{U * 81}", flush=True)
    dZ3 = torch.randn(2, U * 9, 64, device=dev)
    rows = plan.num_windows * 9
    out = torch.empty(2, rows, 64, device=dev)
    t_slot = timeit(lambda: nat.segment_sum(dZ3, part, rows, slot=mb.slot, sub=9, out=out))
    ref = out.clone()
    # compacted: keep entries whose frame is in the minibatch, source row = slot*9 + p3
    s = mb.slot[part.idx.long() // 9]
    keep = s >= 0
    ck = part.key[keep]
    ci = (s[keep].long() * 9 + part.idx[keep].long() % 9)
    cplan = SegmentPlan(ck, ci, part.item_len)
    t_comp = timeit(lambda: nat.segment_sum(dZ3, cplan, rows, out=out))
    print(f"seg_sum slot-list: {t_slot:.1f} us   compacted ({cplan.nnz} entries): {t_comp:.1f} us  "
          f"max|diff| {float((out - ref).abs().max()):.3g}", flush=True)
    gb = cplan.nnz * 512 / 1e9
    print(f"row bytes gathered {gb:.2f} GB -> {gb / (t_comp * 1e-6) / 1e3:.2f} TB/s (compacted)", flush=True)
    for L in (256, 512, 2048, 4096):
        cp = SegmentPlan(ck, ci, L)
        print(f"  compacted item_len {L}: {timeit(lambda: nat.segment_sum(dZ3, cp, rows, out=out)):.1f} us", flush=True)
    # source-sorted order inside each destination already (stable); try a random order within dst
    perm = torch.randperm(ck.numel(), device=dev)
    k2, o2 = torch.sort(ck[perm].long(), stable=True)
    rp = SegmentPlan(k2, ci[perm][o2], part.item_len)
    print(f"  compacted, random order within dst: {timeit(lambda: nat.segment_sum(dZ3, rp, rows, out=out)):.1f} us",
          flush=True)
    # one tower only (half the bytes, table 264 MB)
    d1 = dZ3[:1].contiguous()
    o1 = out[:1].contiguous()
    print(f"  compacted, one tower: {timeit(lambda: nat.segment_sum(d1, cplan, rows, out=o1)):.1f} us", flush=True)
    blocks_probe.ctx = {"ck": ck, "ci": ci, "dZ3": dZ3, "rows": rows, "U": U}
    blocks_probe()


def blocks_probe():
    """Source-blocked compacted lists: block b holds the entries whose minibatch frame u lies in
    the b-th of nb contiguous u ranges (its dZ3 rows: 1/nb of the table), summed block after block
    into dQ (accumulate)."""
    import merlin._native as nat
    from merlin.windows import SegmentPlan
    g = blocks_probe.ctx
    ck, ci, dZ3, rows, U = g["ck"], g["ci"], g["dZ3"], g["rows"], g["U"]
    out = torch.empty(2, rows, 64, device=dZ3.device)
    for nb in (1, 2, 3, 4, 8):
        blk = (ci // 9) * nb // U
        key = blk * rows + ck.long()
        k2, o2 = torch.sort(key, stable=True)
        parts = []
        cnt = torch.bincount(blk, minlength=nb).tolist()
        off = 0
        for b, c in enumerate(cnt):
            parts.append(SegmentPlan(k2[off:off + c] - b * rows, ci[o2[off:off + c]], 1024))
            off += c

        def run():
            for b, p in enumerate(parts):
                nat.segment_sum(dZ3, p, rows, out=out, accumulate=b > 0)
        print(f"  compacted, {nb} source blocks (sequential, accumulate): {timeit(run):.1f} us", flush=True)
        d1 = dZ3[:1].contiguous()
        o1 = out[:1].contiguous()

        def run1():
            for b, p in enumerate(parts):
                nat.segment_sum(d1, p, rows, out=o1, accumulate=b > 0)
        print(f"     one tower: {timeit(run1):.1f} us", flush=True)
        for L in (256, 512, 1024):
            cat = SegmentPlan(k2, ci[o2], L)  # one launch, keys (block, dst): partial rows per block
            part = torch.empty(2, nb * rows, 64, device=dZ3.device)

            def run2():
                nat.segment_sum(dZ3, cat, nb * rows, out=part)
                torch.sum(part.view(2, nb, rows, 64), 1, out=out)
            t = timeit(run2)
            tp = timeit(lambda: nat.segment_sum(dZ3, cat, nb * rows, out=part))
            print(f"     one launch, block-major items, L={L}: {t:.1f} us (segment_sum alone {tp:.1f})", flush=True)


if __name__ == "__main__":
    main()
