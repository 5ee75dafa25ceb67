"""Probe: WindowPlan.__init__ (merlin/windows.py) step by step at the bench state, the stream drained around each
step (the same calls in the same order), median of `reps`.  python scripts/probe_plan_steps.py [warm] [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin.dedup import FrameGroups
from merlin.ppo import PPO
from merlin import windows as W


def plan_steps(codes, fg, mark):
    rep = codes.index_select(0, fg.rep)
    F = int(rep.shape[0])
    cls = W.unpack_classes(rep)
    mark("unpack")
    wk = W.window_keys(cls).reshape(-1).to(torch.int32)
    mark("window_keys")
    uniq, inv = torch.unique(wk, return_inverse=True)
    nw = int(uniq.numel())
    mark("window unique")
    rows = W.window_rows(uniq).contiguous()
    hk, ho = torch.sort(rows.reshape(-1), stable=True)
    W.SegmentPlan(hk, ho // 16)
    mark("hist plan")
    pkeys = W.patch_keys(cls).reshape(-1)
    mark("patch_keys")
    pk, kid = torch.unique(pkeys, return_inverse=True)
    K = int(pk.numel())
    mark("patch unique")
    ks, ko = torch.sort(kid.to(torch.int32), stable=True)
    W.SegmentPlan(ks, ko)
    mark("patch plan")
    pd = W.digits5(pk, 25).view(K, 5, 5)
    bdst, bsrc, wdst, off = [], [], [], 0
    ar = torch.arange(K, dtype=torch.int64, device=codes.device)
    for ky in range(3):
        ub, bid = torch.unique(W.base5(pd[:, ky:ky + 3, :].reshape(K, 15)), return_inverse=True)
        bdst.append(off + bid)
        bsrc.append(ar)
        bd = W.digits5(ub, 15).view(-1, 3, 5)
        for kx in range(3):
            w = torch.searchsorted(uniq, W.base5(bd[:, :, kx:kx + 3].reshape(-1, 9)).to(torch.int32))
            wdst.append((w * 9 + ky * 3 + kx, off + torch.arange(ub.numel(), dtype=torch.int64, device=codes.device)))
        off += int(ub.numel())
    mark("bands")
    bk, bo = torch.sort(torch.cat(bdst).to(torch.int32), stable=True)
    W.SegmentPlan(bk, torch.cat(bsrc)[bo])
    dk, do = torch.sort(torch.cat([d for d, _ in wdst]).to(torch.int32), stable=True)
    W.SegmentPlan(dk, torch.cat([s for _, s in wdst])[do])
    mark("band + dq plans")


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(4096, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, ent_coef=0.05, device=dev)
    for _ in range(warm):
        agent.update(agent.collect_rollouts())
    agent.collect_rollouts()
    codes = agent.buf.flat_codes
    fg = FrameGroups(codes)
    acc = {}
    for _ in range(reps):
        torch.cuda.synchronize()
        last = [time.perf_counter()]

        def mark(name):
            torch.cuda.synchronize()
            t = time.perf_counter()
            acc.setdefault(name, []).append((t - last[0]) * 1e3)
            last[0] = t

        plan_steps(codes, fg, mark)
    print({k: round(statistics.median(v), 2) for k, v in acc.items()}, flush=True)


if __name__ == "__main__":
    main()
