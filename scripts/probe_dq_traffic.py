"""Probe (round 6): what the dQ pass of conv3's backward (k_seg_sum<0, 3>, merlin/fast_step.py _conv3_backward_bulk)
must move at the bench state, against the byte model the bench line divides by.  The model (merlin/_native.py
segment_sum) counts the entry list, every band row of S ONCE and the dQ rows written; but each 3 x 5 row band holds
three 3 x 3 windows (kx = 0, 1, 2), so its S row is the source of three entries, in three different destination
segments -- read three times.  Prints, for one minibatch of the bench rollout (4096 envs x 256 steps after --iters
PPO iterations): the entry count, the live entries (band marked by the S pass), the model's bytes and the bytes of
one read per live entry.
    python scripts/probe_dq_traffic.py [--iters 6]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    args = ap.parse_args()
    from merlin import MerlinVecEnv
    from merlin import _native as nat
    from merlin.dedup import FrameGroups
    from merlin.ppo import PPO
    from merlin.windows import WindowPlan

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
    dY3 = torch.randn(2, U * 9, 64, device=dev)
    Y3 = torch.randn(2, U * 9, 64, device=dev)
    R = nat.segment_sum(dY3, plan.patch_plan, K, slot=mb.slot, sub=9, mask=Y3, fill=False)
    bslot = torch.full((plan.num_bands,), -1, dtype=torch.int32, device=dev)
    nat.segment_sum(R, plan.band_plan, plan.num_bands, slot=kmap, sub=1, fill=False, mark=bslot)
    dq = plan.dq_plan
    nnz = int(dq.nnz)
    live_e = int((bslot.index_select(0, dq.idx[:nnz].long()) >= 0).sum())
    live_b = int((bslot >= 0).sum())
    out_rows = plan.num_windows * 9
    Tw = 2
    model = nnz * 12 + Tw * (plan.num_bands * 256 + out_rows * 256)
    per_entry = nnz * 12 + Tw * (live_e * 256 + out_rows * 256)
    carries = ((nnz + dq.item_len - 1) // dq.item_len) * Tw * 2 * 256
    print(f"U={U} windows={plan.num_windows} bands={plan.num_bands} live bands={live_b} dQ entries={nnz} "
          f"live entries={live_e} ({live_e / max(live_b, 1):.2f} per live band) item_len={dq.item_len}")
    print(f"model bytes (every band row once) {model / 1e6:.1f} MB; one read per live entry {per_entry / 1e6:.1f} MB "
          f"(+ item carries {carries / 1e6:.1f} MB): {per_entry / model:.2f}x the model")


if __name__ == "__main__":
    main()
