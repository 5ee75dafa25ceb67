"""In-process A/B of update-path switches at the bench workload (4096 envs x 256 steps, 10 x 8
minibatches): one agent warmed up to the bench's state, one rollout, then the SAME update (same
weights, optimizer state and minibatch permutations, restored before every run) timed under each
setting in turn, repeatedly -- device-to-device and clock differences between gpurun boxes and the
training state's drift do not enter the comparison.

    python scripts/ab_update.py [repeats] [warmup] [fast,fast_segfix,fast_x6,fast_h3f10_h3d11,...]

Prints ms per update for each setting."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin import _native as nat
from merlin import windows as W
from merlin.ppo import PPO


def main():
    import copy

    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(4096, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=4096 * 256, minibatch_size=4096 * 256 // 8, ent_coef=0.05, device=dev)
    for _ in range(warm):
        agent.update(agent.collect_rollouts())
    lv = agent.collect_rollouts()
    perms = {}

    def fixed_perm(n, epoch):
        if epoch not in perms:
            g = torch.Generator(device=dev)
            g.manual_seed(1000 + epoch)
            perms[epoch] = torch.randperm(n, device=dev, generator=g)
        return perms[epoch]

    agent.perm_fn = fixed_perm
    sd = copy.deepcopy(agent.ac.state_dict())
    opt = copy.deepcopy(agent.optimizer.state_dict())

    clip_adam = agent._clip_adam
    host = {}

    def setter(name):
        def s():
            W.OVERLAP_WGRAD = {"no_overlap": False, "x6_overlap": True}.get(name, "deferred")
            agent.ac.fc1_impl = "hipblaslt" if name == "hipblaslt" else "x6" if "x6" in name else "h3"
            nat.SEG_FUSED = "segfix" not in name  # the segmented sums' fix-ups in a second launch (k_seg_fix)
            nat.H3_NT_CFG["fwd"] = next((int(t[3:]) for t in name.split("_") if t[:3] == "h3f"), 13)
            nat.H3_NT_CFG["dgrad"] = next((int(t[3:]) for t in name.split("_") if t[:3] == "h3d"), 11)
            nat.H3_TN_CFG = next((int(t[3:]) for t in name.split("_") if t[:3] == "h3t"), 0)
            nat.H3_TN_SPLITS = next((int(t[3:]) for t in name.split("_") if t[:3] == "h3s"), 32)
            agent._clip_adam = None if name == "torch_opt" else clip_adam
            agent.fast_step = name.startswith("fast")  # merlin/fast_step.py vs the autograd engine
            from merlin import fast_step as FS

            FS.WGRAD_EARLY = "wgrad_early" in name
            FS.SIDE_PRIORITY = -1 if "sidehi" in name else 0
            FS.SIDE_CU_GROUPS = next((int(t[2:]) for t in name.split("_") if t[:2] == "cu" and t[2:].isdigit()), 0)
            FS.MAIN_PRIORITY = -1 if "mainhi" in name else 0
            FS.WINDOW_H3 = "wh3" in name
            FS.WGRAD_SPLIT_SIDE = "splitside" in name
            FS.PATCH_REUSE = False if "noreuse" in name else "copy" if "reusecopy" in name else "gather"
            nat.H3_HEADS_EPILOGUE = "noheadsepi" not in name
            FS.WGRAD_SIDE = "wgradside" in name  # the weight gradient on a side stream beside conv3's sums
            FS.MASK_COPY_SIDE = "maskside" in name  # the mask-word copy on the side stream
            FS.MASK_ROWS = "maskcopy" not in name  # the mask-word copy instead of the R pass's row map
            FS.DZ_PLANES = "nodzp" not in name  # dz in fp32 (split by the GEMMs) instead of head_bwd's planes
            FS.A3_PLANES = "noa3p" not in name  # a3 in fp32 instead of conv3's planes
            FS.PREFILL = "noprefill" not in name  # conv3's backward fills beside the weight gradient
            FS.WINDOW_BWD_HIP = "nowinbwd" not in name  # the window GEMM's backward on hipBLASLt + torch
            nat.H3_TN_CFG_PLANES = 0 if "tngplanes" in name else 21 if "tq21" in name else 20  # register-staged / 64-row
            nat.H3_NT_CFG["fwd_planes"] = 13 if "ntpgplanes" in name else 60  # the copy-staged forward over planes
            nat.H3_NT_CFG["dgrad_planes"] = next((int(t[3:]) for t in name.split("_") if t[:3] == "h3p"), 62)
            nat.X6_NT_CFG["fwd"] = 28 if "fwd28" in name else 20
            nat.X6_NT_CFG["dgrad"] = 27 if "dgrad27" in name else 22
            nat.X6_TN_CFG = next((int(t[2:]) for t in name.split("_") if t[:2] == "tn" and t[2:].isdigit()), 0)
            nat.X6_TN_SPLITS = 64 if "tn24" in name else next(
                (int(t[1:]) for t in name.split("_") if t[:1] == "s" and t[1:].isdigit()), 32)  # e.g. fast_s64
            if agent.stage_impl != ("torch" if "torch_stage" in name else "hip"):
                agent.stage_impl = "torch" if "torch_stage" in name else "hip"
                agent._wstep = None  # recapture the weight stage with the other table implementation
        return s

    names = sys.argv[3].split(",") if len(sys.argv) > 3 else ["x6_overlap", "no_overlap", "hipblaslt"]
    settings = {n: setter(n) for n in names}
    times = {n: [] for n in settings}
    kt = {}
    for _ in range(iters):
        for n, s in settings.items():
            s()
            agent.ac.load_state_dict(sd)
            agent.optimizer.load_state_dict(opt)
            torch.cuda.synchronize()
            if "_timers" in n:  # bench.py's per-kernel HIP events switched on (_timers4: every 4th launch)
                nat.KernelTimer.start(every=4 if n.endswith("_timers4") else 1)
            t0 = time.perf_counter()
            agent.update(lv)
            torch.cuda.synchronize()
            recs = nat.KernelTimer.stop()
            if recs:  # per-kernel HIP-event times of this run (the last repeat's are printed)
                agg = {}
                for name_, e0, e1, _, _ in recs:
                    a = agg.setdefault(name_, [0, 0.0])
                    a[0] += 1
                    a[1] += e0.elapsed_time(e1)
                kt[n] = agg
            times[n].append((time.perf_counter() - t0) * 1e3)
            host.setdefault(n, []).append(agent.last_host_loop_ms)
    for n, t in times.items():
        t = sorted(t)
        h = sorted(host[n])
        print(f"{n:12s} median {t[len(t) // 2]:.1f} ms/update  min {t[0]:.1f}  all {[round(x, 1) for x in times[n]]}"
              f"  host queueing median {h[len(h) // 2]:.1f} ms")
    print("distinct frames per sample", agent.last_distinct_frac)
    for n, agg in kt.items():
        print(f"-- {n}: per-kernel HIP events (launches, total ms, avg us)")
        for name_, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:16]:
            print(f"   {name_:28s} {c:5d} {ms:9.2f} {ms / c * 1e3:9.1f}")


if __name__ == "__main__":
    main()
