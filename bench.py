#!/usr/bin/env python
"""bench.py -- BASELINE.json metric: env-steps/sec (rollout + GAE + PPO update),
4096 envs per GPU, 16x16 mediumhard (configs[1]; configs[2] when launched on 8 ranks).

One "step" = one PPO iteration of the reference loop (src/ppo.py:64-168) over the
vectorised envs: reset all envs, T=256 env steps x N envs of act -> env-step (HIP),
GAE + whole-batch advantage normalisation (HIP), then 10 epochs x 8 minibatches of
N*T/8 with clip_grad_norm_(0.5) + Adam (PyTorch-ROCm fp32, the reference's precision).
ppo_train.py defaults otherwise (lr 3e-4, gamma .99, lam .95, clip .2, vf .5, ent .05).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank r owns envs [r*N, (r+1)*N) seeded 777 + global index (weak scaling); the update
all-reduces the f32 gradient once per optimizer step and the advantage moments once
per iteration over RCCL.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import glob

import numpy as np
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
# MIOpen: heuristic ("immediate") solver choice instead of a per-shape Find that compiles and
# times every candidate kernel (minutes per new batch shape on a fresh box).  Startup-only
# setting; the convolutions computed are the same fp32 convolutions.
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
os.environ.setdefault("MIOPEN_LOG_LEVEL", "3")

# Algorithmic work per unit: each hand-written kernel's bytes per launch are
# recorded by merlin._native.KernelTimer next to its HIP events (k_env_step: 168 B per
# env-step; k_conv2_lut_fwd: 12,840 B per frame; ...).
# Reference formulation, per env-step: rollout forward of both towers 9.94 MFLOP
#   + 10 epochs x fwd+bwd 25.67 MFLOP (conv1 needs no input gradient) = 266.6 MFLOP.
FWD_MACS = 2 * (1_038_336 + 819_200 + 331_776 + 294_912) + 512 * 3 + 512
BWD_MACS = 2 * FWD_MACS - 2 * 1_038_336
# What this implementation runs on the matrix/vector FP32 units: conv1+conv2 are table
# lookups (no MACs); per rollout frame fc1 + heads of both towers, and per rollout conv3's
# all-windows table (one [5^9, 64] x [64, 576] product per tower, merlin/actor_critic.py
# rollout_pack); in the update fc1 + heads run once per distinct frame of a minibatch
# (merlin/dedup.py) and conv3 once per distinct receptive-field window of the rollout
# (merlin/windows.py: the [windows, 64] x [64, 576] product per tower); backward = input grad +
# weight grad (2x).
GEMM_FWD_MACS = 2 * (331_776 + 294_912) + 512 * 3 + 512  # the per-frame formulation (no windows)
ROLLOUT_TABLE_MACS = 2 * (4 ** 9 + 3 * 4 ** 8) * 64 * 576  # per rollout (the acting table's compact keys)
FC_FWD_MACS = 2 * 294_912 + 512 * 3 + 512
WINDOW_FWD_MACS = 2 * 64 * 576  # per window per minibatch
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3  # MI355X dense FP32 (vector == f32 MFMA rate)
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense BF16 MFMA (MI355X_MICROARCH.md; no sparsity)
# fc1's three GEMMs run on the matrix cores in plane form: "h3" (default, csrc/merlin_h3.hip) three f16 MFMA
# products per fp32 product, "x6" (csrc/merlin_gemm.hip) six bf16 products; their executed MFMA work is that
# multiple of the fp32 FLOP count, priced against the dense 16-bit MFMA peak (f16 = bf16 rate)
X6_GEMMS = ("gemm_fc1_fwd", "gemm_fc1_dgrad", "gemm_wgrad")
PLANE_PRODUCTS = {"h3": 3, "x6": 6}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--k-steps", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--minibatches", type=int, default=8)
    ap.add_argument("--difficulty", default="mediumhard")
    ap.add_argument("--size", type=int, default=16)
    ap.add_argument("--timer-every", type=int, default=4,
                    help="HIP-event timing of every k-th launch of each kernel in the timed region (kernels table, "
                         "rooflines); the event records cost the loop ~2-3 %% when every launch is timed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-tiers", action="store_true")
    ap.add_argument("--env-tier-only", action="store_true",
                    help="only the HBM-scale env tier (2M envs; for the k_env_step rocprofv3 --pmc pass)")
    ap.add_argument("--no-dedup", action="store_true",
                    help="evaluate the towers on every minibatch sample (no distinct-frame grouping)")
    ap.add_argument("--no-windows", action="store_true",
                    help="conv2/conv3 per (frame, position) table lookups instead of per distinct window")
    ap.add_argument("--no-graph", action="store_true", help="launch the rollout eagerly (no captured HIP graph)")
    ap.add_argument("--fomaml", action="store_true",
                    help="cfg 5 instead: FOMAML meta-iterations, tasks_per_batch=32 x k_steps=256")
    ap.add_argument("--tasks", type=int, default=32)
    return ap.parse_args()


def fomaml_bench(args):
    """BASELINE cfg 5: one meta-iteration = 32 tasks x (256 support + 256 query) env steps,
    inner SGD step per task, meta Adam step (merlin.fomaml, batched over tasks)."""
    import torch

    from merlin import ScenarioCreator
    from merlin.fomaml import FOMAML

    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    fm = FOMAML(ScenarioCreator(), lr_inner=0.01, lr_outer=3e-4, device=dev, difficulty=args.difficulty)
    rs = np.random.RandomState(42)
    seeds = lambda: rs.choice(100000, args.tasks, replace=False)  # noqa: E731
    for _ in range(args.warmup):
        fm.meta_train_step(seeds(), k_support=args.k_steps, k_query=args.k_steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fm.meta_train_step(seeds(), k_support=args.k_steps, k_query=args.k_steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = args.steps * args.tasks * 2 * args.k_steps
    print(json.dumps({"metric": "FOMAML env-steps/sec (support+query rollouts, inner SGD, meta Adam)",
                      "value": round(steps / el, 1), "unit": "env-steps/s", "n_gpus": 1, "steps": args.steps,
                      "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 2),
                      "higher_is_better": True, "dtype": "fp32", "data": "synthetic",
                      "config": {"workload": f"FOMAML {args.difficulty} tasks_per_batch={args.tasks} "
                                             f"k_steps={args.k_steps}"}}), flush=True)


def wgrad_side() -> bool:
    from merlin import fast_step as FS

    return bool(FS.WGRAD_SIDE)


def fomaml_tier(device, difficulty, tasks=32, k=256, warmup=3, steps=4):
    """BASELINE cfg 5 inside the default run: meta-iterations of 32 tasks x (256 support + 256
    query) env steps with the inner SGD step and the meta Adam step (merlin.fomaml, batched over
    tasks); env-steps/s of the meta step, after `warmup` meta steps (the first two run eagerly, the third records
    the inner / outer graphs: merlin.fomaml CAPTURE_AFTER)."""
    import torch

    from merlin import ScenarioCreator
    from merlin.fomaml import FOMAML

    torch.manual_seed(42)
    fm = FOMAML(ScenarioCreator(), lr_inner=0.01, lr_outer=3e-4, device=device, difficulty=difficulty)
    rs = np.random.RandomState(42)
    for _ in range(warmup):
        fm.meta_train_step(rs.choice(100000, tasks, replace=False), k_support=k, k_query=k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fm.meta_train_step(rs.choice(100000, tasks, replace=False), k_support=k, k_query=k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(steps * tasks * 2 * k / el, 1), "unit": "env-steps/s", "ms_per_meta_step":
            round(el / steps * 1e3, 1), "config": f"tasks_per_batch={tasks} k_support=k_query={k}, {difficulty}"}


def env_only_tier(torch, MerlinVecEnv, n, T, difficulty, size, device):
    """Tier E: env dynamics + obs codes only, actions pre-generated.
    (a) one launch steps all T steps with state on chip; (b) T single-step launches."""
    env = MerlinVecEnv(n, difficulty=difficulty, size=size, seed=4242, device=device)
    env.reset()
    g = torch.Generator(device=device)
    g.manual_seed(7)
    acts = torch.randint(0, 3, (T, n), device=device, generator=g)
    obs = torch.empty((T, n, 8), dtype=torch.int32, device=device)
    rew = torch.empty((T, n), dtype=torch.float32, device=device)
    done = torch.empty((T, n), dtype=torch.float32, device=device)
    for _ in range(2):
        env.step_into(acts, obs, rew, None, None, done, n_steps=T, action_stride=n)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        env.step_into(acts, obs, rew, None, None, done, n_steps=T, action_stride=n)
    e1.record()
    torch.cuda.synchronize()
    fused = reps * T * n / (e0.elapsed_time(e1) / 1e3)
    e0.record()
    for t in range(T):
        env.step_into(acts[t], obs[t], rew[t], None, None, done[t])
    e1.record()
    torch.cuda.synchronize()
    single = T * n / (e0.elapsed_time(e1) / 1e3)
    env.errors()
    env.close()
    return fused, single


def env_large_tier(torch, MerlinVecEnv, difficulty, size, device, n=1 << 21, T=16):
    """Tier E at HBM scale: 2M envs (0.35 GB of env state and outputs per step),
    T single-step launches on pre-generated actions, 168 algorithmic bytes per env-step
    (merlin.envs.ENV_STEP_BYTES); at the bench's 4096 envs the kernel is latency-bound (64 waves on
    256 CUs), here it streams.  Two timings of the same T steps:
      roofline   k_env_step alone (autoreset off: no resets, nothing else launched) -> HBM fraction;
      with_resets  auto-reset on: each launch is k_env_step + k_env_fallback (the resets whose
                 look-ahead map slot was already used since the last refill -- at 2M envs some every
                 step, each a one-thread map generation of tens of microseconds) + k_env_refill every
                 16 launches (T = 16 = one refill inside the timed steps)."""
    from merlin.envs import ENV_STEP_BYTES

    env = MerlinVecEnv(n, difficulty=difficulty, size=size, seed=31337, device=device)
    env.reset()
    g = torch.Generator(device=device)
    g.manual_seed(9)
    acts = torch.randint(0, 3, (T, n), device=device, generator=g)
    obs = torch.empty((T, n, 8), dtype=torch.int32, device=device)
    rew = torch.empty((T, n), dtype=torch.float32, device=device)
    done = torch.empty((T, n), dtype=torch.float32, device=device)
    env.step_into(acts[0], obs[0], rew[0], None, None, done[0])
    torch.cuda.synchronize()

    def timed(autoreset):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(T):
            env.step_into(acts[t], obs[t], rew[t], None, None, done[t], autoreset=autoreset)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3

    sec_reset = timed(True)
    resets = int(done.sum())
    sec = timed(False)  # truncated envs stay done (no reset): same bytes per env-step
    env.errors()
    env.close()
    rate = T * n / sec
    gbs = rate * ENV_STEP_BYTES / 1e9
    return {"kernel": "k_env_step", "num_envs": n, "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("k_env_step_large"),
            "env_steps_per_s": round(rate, 1), "bytes_per_launch": n * ENV_STEP_BYTES,
            "avg_launch_us": round(sec / T * 1e6, 2), "launches": T,
            "with_resets": {"env_steps_per_s": round(T * n / sec_reset, 1),
                            "us_per_step": round(sec_reset / T * 1e6, 2), "resets": resets}}


def x6_standalone(torch, U, device, impl="h3", reps=10):
    """fc1's three plane-form GEMMs timed alone (HIP events, no other stream active) at the update's shape
    (U distinct frames per minibatch): in the timed loop the weight gradient shares the chip with
    conv3's backward sums on the other stream, so its in-loop event time includes that sharing."""
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(0)
    a3 = torch.relu(torch.randn(2, U, 576, device=device, generator=g))
    dz = torch.randn(2, U, 512, device=device, generator=g) * 1e-6
    W = torch.randn(2, 512, 576, device=device, generator=g) / 24
    Wt = W.transpose(1, 2).contiguous()
    b = torch.zeros(2, 512, device=device)
    if impl == "h3":
        from merlin import fast_step as FS

        am3, amz, amW = nat.h3_amax(a3), nat.h3_amax(dz), nat.h3_amax(W)
        Wp, Wtp = nat.h3_split(W, amW), nat.h3_split(Wt, amW)
        # the update's forms: a3 read through a row map (here the identity), dz as planes (DZ_PLANES: the
        # plane-operand input gradient, the weight gradient staging dz's planes as copies)
        rows = torch.arange(U * 9, dtype=torch.int32, device=device)
        dzo = nat.h3_split(dz, amz) if FS.DZ_PLANES else dz
        a3p = FS.DZ_PLANES and FS.A3_PLANES  # a3 as planes too: the forward stages copies, the LDS-DMA TN
        a3o = nat.h3_split(a3, am3) if a3p else a3
        Wa = torch.randn(3, 512, device=device, generator=g) / 24
        Wc = torch.randn(1, 512, device=device, generator=g) / 24
        dgrad = ((lambda: nat.h3_gemm_nt_planes(dzo, amz, Wtp, amW, cfg=nat.H3_NT_CFG["dgrad_planes"]))
                 if FS.DZ_PLANES else (lambda: nat.h3_gemm_nt(dz, amz, Wtp, amW, cfg=nat.H3_NT_CFG["dgrad"])))
        fcfg = nat.H3_NT_CFG["fwd_planes" if a3p else "fwd"]
        runs = {"gemm_fc1_fwd": lambda: nat.h3_gemm_nt_heads(a3o, am3, Wp, amW, b, Wa, Wc, cfg=fcfg, rows=rows),
                "gemm_fc1_dgrad": dgrad,
                "gemm_wgrad": lambda: nat.h3_gemm_tn(dzo, amz, a3o, am3, rows=rows,
                                                     cfg=nat.H3_TN_CFG_PLANES if a3p else None)}
    else:
        Wp, Wtp = nat.x6_split(W), nat.x6_split(Wt)
        runs = {"gemm_fc1_fwd": lambda: nat.x6_gemm_nt(a3, Wp, bias=b, cfg=nat.X6_NT_CFG["fwd"]),
                "gemm_fc1_dgrad": lambda: nat.x6_gemm_nt(dz, Wtp, cfg=nat.X6_NT_CFG["dgrad"]),
                "gemm_wgrad": lambda: nat.x6_gemm_tn(dz, a3)}
    P = PLANE_PRODUCTS[impl]
    out = {}
    for name, fn in runs.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        ex = P * 2 * 2 * U * 576 * 512 / (us * 1e-6) / 1e12
        out[name] = {"avg_launch_us": round(us, 2), "achieved": round(ex, 2), "peak": BF16_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(ex / BF16_PEAK_TFLOPS, 4),
                     "fp32_equivalent_tflops": round(ex / P, 2)}
    return {"rows": U, "impl": impl, "kernels": out}


def cpu_baseline():
    """The oracle's CPU port of the reference loop (oracle/ppo_cpu.py), N=1 env, batch 2048, 10 epochs x
    8 minibatches of 256, plus the per-iteration 3-episode deterministic eval of ppo/ppo_train.py:150
    (BASELINE.md's plan: counted env-steps / wall time without and with the eval; all host threads and
    1 thread).  One iteration per thread count (~10 s with all threads, ~20-40 s on one)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch

    import ppo_cpu  # noqa: E402  (baseline leg only)

    threads = torch.get_num_threads()
    steps, secs, secs_eval = ppo_cpu.run_iterations(n_iter=1, eval_episodes=3)
    torch.set_num_threads(1)
    try:
        s1, t1, t1e = ppo_cpu.run_iterations(n_iter=1, eval_episodes=3)
    finally:
        torch.set_num_threads(threads)
    return {"value": round(steps / secs, 2), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "value_with_eval": round(steps / secs_eval, 2),
            "one_thread": {"value": round(s1 / t1, 2), "value_with_eval": round(s1 / t1e, 2), "cores": 1},
            "sample": "1 PPO iteration of the reference loop on CPU per thread count: 1 mediumhard 16x16 env "
                      "(C oracle + RGB render), batch 2048, 10 epochs x 8 minibatches of 256, fp32 torch CNN "
                      "(cfg 1 shape); value_with_eval adds the 3-episode deterministic eval of "
                      "ppo/ppo_train.py:150"}


# bench names -> rocprofv3 kernel names (untruncated: template arguments kept).  A span made of several
# kernels adds their bytes; the first name of a tuple must be present, the rest (e.g. a segmented sum's
# fix-up pass, absent when no destination crosses an item) count when they are.
PMC_ALIAS = {"k_seg_sum_R": ("k_seg_sum<3, 1>",),  # the R pass reading each row's mask word through its representative
             "k_seg_sum_S": ("k_seg_sum<0, 2>",),
             "k_seg_sum_dQ": ("k_seg_sum<0, 3>",),
             "k_seg_sum_dT2": ("k_seg_sum<0, 4>",),
             "k_window_lut": ("k_window_lut<0>",),
             "k_window_lut_all": ("k_window_lut<1>",)}
# with conv3's patch reuse (merlin/fast_step.py PATCH_REUSE = "gather") the update's k_window_conv3 span is the
# representatives' kernel + the mask-word copy, and fc1's forward / weight gradient read a3 through the row map
PMC_ALIAS_GATHER = {"k_window_conv3": ("k_window_conv3_reps", "k_window_conv3_copy<false>", "k_q_colmax", "k_q_bound")}
# rocprofv3 names of merlin_h3_gemm_nt's configurations (csrc/merlin_h3.hip launch_h3_gemm_nt)
H3_NT_NAMES = {0: "k_h3_nt<256, 128, 4, 2, {}>", 1: "k_h3_nt<128, 192, 4, 2, {}>", 2: "k_h3_nt<128, 128, 2, 2, {}>",
               3: "k_h3_nt<128, 256, 2, 4, {}>", 10: "k_h3_ntp<256, 128, 4, 2, {}>", 11: "k_h3_ntp<128, 192, 4, 2, {}>",
               12: "k_h3_ntp<128, 128, 2, 2, {}>", 13: "k_h3_ntp<128, 256, 2, 4, {}>"}


def h3_gemm_names(nat):
    """PMC_ALIAS entries of the update's fc1 forward (bias + ReLU epilogue) and input gradient (and, with the patch
    reuse's gathered rows, of conv3 and the weight gradient)."""
    from merlin import fast_step as FS

    heads = nat.H3_HEADS_EPILOGUE and nat.lib().merlin_h3_heads_parts(512, nat.H3_NT_CFG["fwd"]) > 0
    fwd = H3_NT_NAMES.get(nat.H3_NT_CFG["fwd"], "?").format(2 if heads else 1)  # EPI 2: the heads in the epilogue
    out = {"gemm_fc1_dgrad": (H3_NT_NAMES.get(nat.H3_NT_CFG["dgrad"], "?").format(0),)}
    if not FS.WINDOW_H3 and FS.WINDOW_BWD_HIP:  # conv3's per-window GEMM on the exact-f32 kernel (_native.window_gemm_fwd)
        out["gemm_window_fwd"] = ("k_winfwd",)
    dzp = FS.DZ_PLANES and FS.PATCH_REUSE == "gather"
    if dzp:  # dz leaves the heads' backward as planes: the input gradient on the plane-operand DMA kernel (cfg 62)
        out["gemm_fc1_dgrad"] = ("k_h3_pq<128, 192, 4, 2, 0, 16>",)
    out["k_head_bwd"] = (f"k_head_bwd<3, {'true' if dzp else 'false'}>", "k_head_fold")
    if heads:
        out["k_heads_fwd"] = ("k_heads_combine",)
    if nat.H3_HEADS_EPILOGUE and nat.lib().merlin_h3_heads_parts(512, nat.H3_NT_CFG["rollout"]) > 0:
        # the acting GEMM with the heads only in its epilogue (EPI 3) and the draw from its partials
        out["gemm_rollout_fc1"] = (H3_NT_NAMES.get(nat.H3_NT_CFG["rollout"], "?").format(3),)
        out["k_act_heads"] = ("k_act_draw",)
    if FS.PATCH_REUSE == "gather":
        a3p = dzp and FS.A3_PLANES
        wg = (f"k_h3_tq<128, 192, 4, 2>" if a3p and nat.H3_TN_CFG_PLANES == 20 else
              f"k_h3_tng<128, 192, 4, 2, {'true' if dzp else 'false'}, {'true' if a3p else 'false'}>")
        fw = ("k_h3_pqg<128, 256, 2, 4, 2>" if a3p and nat.H3_NT_CFG["fwd_planes"] == 60 else
              fwd.replace("k_h3_ntp<", "k_h3_ntpg<").replace(">", ", true>" if a3p else ", false>"))
        return {**out, **PMC_ALIAS_GATHER, "gemm_wgrad": (wg, "k_x6_fold"), "gemm_fc1_fwd": (fw,)}
    return {**out, "gemm_fc1_fwd": (fwd,)}
PMC_FILE = os.environ.get("MERLIN_PMC_FILE")  # default: the newest profiles/*_pmc.json holding the kernel


def pmc_traffic(kernel: str):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 --pmc passes of the same bench
    command (profiles/*_pmc.json: FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM + WRITE_SIZE);
    a span made of several kernels (PMC_ALIAS tuple) adds theirs."""
    from merlin import _native as nat

    names = {**PMC_ALIAS, **h3_gemm_names(nat)}.get(kernel, kernel)
    names = names if isinstance(names, tuple) else (names,)
    files = [PMC_FILE] if PMC_FILE else sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")), reverse=True)
    if not PMC_FILE:
        # only PMC passes at least as new as the newest kernel trace (profile names start with their round tag,
        # e.g. r05j_): an older pass measured other code, and a kernel it holds under the same name is not this one
        stats = sorted(glob.glob(os.path.join(REPO, "profiles", "*_kernel_stats.md")))
        newest = os.path.basename(stats[-1]).split("_")[0] if stats else ""
        files = [f for f in files if os.path.basename(f).split("_")[0] >= newest]
    def entry(dd, n):  # the exact name, else the one kernel whose template arguments extend the alias's
        if n in dd or not n.endswith(">"):
            return dd.get(n, {})
        ext = [k for k in dd if k.startswith(n[:-1] + ",")]
        return dd[ext[0]] if len(ext) == 1 else {}

    for f in files:
        try:
            dd = json.load(open(f))
        except Exception:
            continue
        got = [entry(dd, n).get("hbm_bytes_per_launch") for n in names]
        if got[0]:
            return int(sum(g for g in got if g))
    return None


def gather_note(name, k):
    """k_window_conv3 reads little HBM: every computed output row sums 9 rows of the per-minibatch Q table (~15 MB
    per tower, L2 / Infinity-Cache resident), so its bound is the cache gather rate (MI355X_MICROARCH.md 'Indexed
    rows': 16.8-18.8 TB/s for L2-resident rows), not HBM.  bytes_per_launch counts the rows written (with the patch
    reuse: the representatives', 256 + 8 B per row and tower), so 9 x that is the Q-row gather."""
    if name != "k_window_conv3":
        return {}
    gathered = 9 * k["bytes_per_launch"]  # ~ 9 Q rows of 256 B per written Y3 row
    tbs = gathered / (k["avg_us"] * 1e-6) / 1e12
    return {"cache_gather": {"bytes_per_launch": gathered, "achieved_tbs": round(tbs, 2),
                             "guide_l2_gather_tbs": [16.8, 18.8], "frac_of_18_8": round(tbs / 18.8, 3)}}


def kernel_table(records, counts=None):
    """{name: launches, total ms, avg us, algorithmic bytes (GB/s) or flops (TFLOP/s) per launch}
    from HIP events; `counts` = every launch of each name in the region (KernelTimer.counts): when only
    each every-th launch was timed (`launches_timed` < launches), total_ms = the timed average x the true
    launch count."""
    agg = {}
    for name, e0, e1, nbytes, flops in records:
        ms = e0.elapsed_time(e1)
        a = agg.setdefault(name, [0, 0.0, 0, 0])
        a[0] += 1
        a[1] += ms
        a[2] += nbytes
        a[3] += flops
    out = {}
    for name, (cnt, ms, nb, fl) in agg.items():
        n = int(counts.get(name, cnt)) if counts else cnt
        d = {"launches": n, "total_ms": round(ms / cnt * n, 3), "avg_us": round(ms / cnt * 1e3, 2)}
        if n != cnt:
            d["launches_timed"] = cnt
        if fl:
            d.update(flops_per_launch=fl // cnt, tflops=round(fl / (ms / 1e3) / 1e12, 2))
        else:
            d.update(bytes_per_launch=nb // cnt, gbs=round(nb / (ms / 1e3) / 1e9, 2))
        out[name] = d
    return out


# the MFMA each plane-form GEMM runs on (merlin._native.H3_* / X6_NT_CFG / X6_TN_CFG)
PLANE_MFMA = {"h3": "f16 32x32x16", "x6": "bf16 32x32x16 (forward / input gradient), 16x16x32 (weight gradient)"}


def plane_impl(name):
    """'h3' / 'x6' when the span `name` was timed through that plane-form GEMM wrapper (merlin._native.H3_SPANS /
    X6_SPANS), else None (a hipBLASLt fp32 GEMM)."""
    from merlin import _native as nat

    return "h3" if name in nat.H3_SPANS else "x6" if name in nat.X6_SPANS else None


def roofline_of(name, k, impl=None):
    traffic = pmc_traffic(name)
    impl = plane_impl(name) if "tflops" in k else None
    if impl is not None:  # fp32 products on the 16-bit matrix cores in plane form
        P = PLANE_PRODUCTS[impl]
        ex = k["tflops"] * P
        return {"kernel": name, "bound": "mfma", "achieved": round(ex, 2), "peak": BF16_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ex / BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                "flops_per_launch": k["flops_per_launch"] * P, "avg_launch_us": k["avg_us"],
                "launches": k["launches"], "mfma": f"{PLANE_MFMA[impl]}, {P} plane products per fp32 product",
                # the same rate counted in fp32 products, against the ceiling of the instructions that run
                # (dense 16-bit MFMA peak / plane products); frac equals the executed-MFMA frac above
                "fp32_equivalent": {"achieved": k["tflops"], "ceiling": round(BF16_PEAK_TFLOPS / P, 1),
                                    "unit": "TFLOP/s (fp32 products)"}}
    if "tflops" in k:  # a hipBLASLt GEMM: f32 MFMA bound
        return {"kernel": name, "bound": "mfma", "achieved": k["tflops"], "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(k["tflops"] / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                "flops_per_launch": k["flops_per_launch"], "avg_launch_us": k["avg_us"], "launches": k["launches"]}
    return {"kernel": name, "bound": "hbm", "achieved": k["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(k["gbs"] / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": k["bytes_per_launch"], "avg_launch_us": k["avg_us"], "launches": k["launches"]}


def _median_iter_rate(agent, warmup, iters):
    """env-steps/s of rollout + update: `warmup` untimed iterations, then the median of `iters` iterations
    each timed on its own (host clock around a synchronised iteration)."""
    import torch

    for _ in range(warmup):
        agent.update(agent.collect_rollouts())
    times = []
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        agent.update(agent.collect_rollouts())
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return agent.batch_size / float(np.median(times)), times


def floor_tier(agent, warmup=1, iters=3):
    """The update without exploiting repeated observations, on the agent's current state, after the timed
    region: env-steps/s of rollout + update, median of `iters` iterations after `warmup` untimed ones per
    setting (the first iteration of a setting pays its one-time costs: MIOpen / hipBLASLt heuristics for
    new shapes, allocator growth).
      no_windows           distinct frames per minibatch (merlin/dedup.py), conv1+conv2 by per-position
                           table lookups and conv3 as an im2col GEMM per distinct frame
      no_dedup_no_windows  the same on every minibatch sample (no grouping at all)
    Without the windows the grouping's gain is only the distinct fraction of the sample count (0.89 at
    the bench state) while it adds a sort + gather per minibatch, so the two floors are close."""
    saved = (agent.dedup, agent.windows)
    out = {}
    try:
        for name, (dedup, windows) in (("no_windows", (True, False)), ("no_dedup_no_windows", (False, False))):
            agent.dedup, agent.windows = dedup, windows
            rate, times = _median_iter_rate(agent, warmup, iters)
            out[name] = round(rate, 1)
            out[name + "_iter_ms"] = [round(t * 1e3, 1) for t in times]
    finally:
        agent.dedup, agent.windows = saved
    return out


def hard22_tier(device, N, T, epochs, minibatches, warmup=2, iters=3):
    """BASELINE cfg 4: the same full loop on hard 22x22 grids (src/custom_envs/hard_env.py:11-97: mid
    wall with 2-5 gaps, 6-12 extra walls, goal in the right half), 4096 envs x 256 steps, a fresh agent
    (torch seed 777, env seeds 777+i); median of `iters` iterations after `warmup`."""
    import torch

    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    # the tiers before this one leave blocks in torch's caching allocator: release them, so the acting path's
    # free-memory check (CNNActorCritic._use_all_windows, 12 GB for the all-windows table) sees the device as the main
    # loop did
    torch.cuda.empty_cache()
    env = MerlinVecEnv(N, difficulty="hard", size=22, seed=777, device=device)
    torch.manual_seed(777)
    agent = PPO(env, lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=epochs, batch_size=N * T,
                minibatch_size=N * T // minibatches, vf_coef=0.5, ent_coef=0.05, device=device)
    rate, times = _median_iter_rate(agent, warmup, iters)
    out = {"value": round(rate, 1), "unit": "env-steps/s", "iter_ms": [round(t * 1e3, 1) for t in times],
           "config": f"hard 22x22, {N} envs x k_steps {T}, {epochs} epochs x {minibatches} minibatches",
           "state": f"iterations {warmup + 1}..{warmup + iters} from random init",
           "distinct_frames_per_sample": round(agent.last_distinct_frac, 4),
           "windows_per_update": agent.last_num_windows,
           "rollout_acting": "all-windows conv3 table" if agent.rollout_all_windows else "per-frame conv2 lookups"}
    # the data-independent floor of this tier too (round-5 verdict): the same loop with neither the distinct-frame
    # grouping nor the windows, on the agent's current state
    saved = (agent.dedup, agent.windows)
    try:
        agent.dedup, agent.windows = False, False
        frate, ftimes = _median_iter_rate(agent, 1, 2)
        out["full_loop_floor"] = {"no_dedup_no_windows": round(frate, 1),
                                  "no_dedup_no_windows_iter_ms": [round(t * 1e3, 1) for t in ftimes]}
    finally:
        agent.dedup, agent.windows = saved
    env.close()
    del agent
    torch.cuda.empty_cache()
    return out


def rollout_ms_of(ph):
    return sum(a.elapsed_time(b) for a, b, _ in ph) / len(ph)


def update_ms_of(ph):
    return sum(b.elapsed_time(c) for _, b, c in ph) / len(ph)


def heartbeat(state):
    import threading

    def run():
        t0 = time.time()
        while True:
            time.sleep(45)
            print(f"[bench] alive {time.time() - t0:.0f}s phase={state.get('phase')}", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    state = {"phase": "init"}
    heartbeat(state)
    if args.fomaml:
        return fomaml_bench(args)
    import torch
    import torch.distributed as dist

    from merlin import MerlinVecEnv
    if args.env_tier_only:
        torch.cuda.set_device(0)
        print(json.dumps(env_large_tier(torch, MerlinVecEnv, args.difficulty, args.size, torch.device("cuda", 0))),
              flush=True)
        return
    from merlin import _native as nat
    from merlin.distributed import DataParallel
    from merlin.ppo import PPO

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one GPU per rank (LOCAL_RANK); MERLIN_BENCH_DEVICE pins every rank to one device and
    # MERLIN_DIST_BACKEND=gloo replaces RCCL, so a world-2 run can rehearse the multi-rank path on
    # one GPU (tests/test_gpu_bench_dp.py: RCCL needs one GPU per rank)
    local = int(os.environ.get("MERLIN_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    backend = os.environ.get("MERLIN_DIST_BACKEND", "nccl") if world > 1 else None
    dp = DataParallel.init_from_env(backend, device)
    # small host-side exchanges (timing, per-rank spread) on the backend's own device kind
    coll_dev = device if (backend or "nccl") == "nccl" else torch.device("cpu")

    N, T = args.num_envs, args.k_steps
    B = N * T
    env = MerlinVecEnv(N, difficulty=args.difficulty, size=args.size, seed=777, device=device,
                       env_offset=rank * N)
    torch.manual_seed(777)
    agent = PPO(env, lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=args.epochs, batch_size=B,
                minibatch_size=B // args.minibatches, vf_coef=0.5, ent_coef=0.05, device=device, dp=dp,
                dedup=not args.no_dedup, windows=not args.no_windows, rollout_graph=not args.no_graph)

    state["phase"] = "warmup"
    for _ in range(args.warmup):
        agent.update(agent.collect_rollouts())
    torch.cuda.synchronize()
    if dp.enabled:
        dist.barrier()

    state["phase"] = "timed"
    nat.KernelTimer.start(every=args.timer_every)
    ph = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        lv = agent.collect_rollouts()
        e1.record()
        agent.update(lv)
        e2.record()
        ph.append((e0, e1, e2))
    torch.cuda.synchronize()
    if dp.enabled:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dp.enabled:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kernels = kernel_table(nat.KernelTimer.stop(), dict(nat.KernelTimer.counts))
    rollout_ms, update_ms = rollout_ms_of(ph), update_ms_of(ph)
    value = args.steps * B * world / elapsed
    rank_spread = None
    if dp.enabled:
        # per-rank work of the timed iterations: the gradient all-reduce of every optimizer step makes
        # all ranks wait for the slowest, so the imbalance shows as each rank's own GPU-kernel time (HIP
        # event spans of the timed kernels) and its distinct frames per sample (the update's work
        # scales with them), not in the phase times, which the all-reduce equalises
        busy = sum(k["total_ms"] for k in kernels.values()) / args.steps
        mine = torch.tensor([rollout_ms_of(ph), update_ms_of(ph), busy,
                             agent.last_distinct_frac if agent.last_distinct_frac is not None else 1.0],
                            dtype=torch.float64, device=coll_dev)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        a = torch.stack(allv).cpu().numpy()
        rank_spread = {"rollout_ms": [round(float(x), 2) for x in a[:, 0]],
                       "update_ms": [round(float(x), 2) for x in a[:, 1]],
                       "kernel_ms_per_iter": [round(float(x), 2) for x in a[:, 2]],
                       "distinct_frames_per_sample": [round(float(x), 4) for x in a[:, 3]],
                       "kernel_ms_max_over_min": round(float(a[:, 2].max() / max(a[:, 2].min(), 1e-9)), 4)}
        # the last collective of the run: everything below is rank 0 alone and collective-free (the tiers,
        # which build agents whose updates all-reduce, run only at world 1; the N=1 line carries them)
        dist.barrier()
        if rank != 0:
            dist.destroy_process_group()
            return
    dominant = max(kernels, key=lambda k: kernels[k]["total_ms"])
    fc1 = getattr(agent.ac, "fc1_impl", None)
    x6 = fc1 in PLANE_PRODUCTS
    handwritten = max((k for k in kernels if k.startswith("k_")), key=lambda k: kernels[k]["total_ms"])
    ref_flop_per_step = 2 * FWD_MACS + args.epochs * 2 * (FWD_MACS + BWD_MACS)
    frac = agent.last_distinct_frac if agent.last_distinct_frac is not None else 1.0
    if agent.last_num_windows is not None:
        upd = 3 * args.epochs * (FC_FWD_MACS * frac + WINDOW_FWD_MACS * agent.last_num_windows * args.minibatches / B)
    else:
        upd = 3 * args.epochs * GEMM_FWD_MACS * frac
    exec_flop_per_step = 2 * (FC_FWD_MACS + ROLLOUT_TABLE_MACS / B + upd)
    loop_tflops = value / world * exec_flop_per_step / 1e12
    loop_peak = round(BF16_PEAK_TFLOPS / PLANE_PRODUCTS[fc1], 1) if x6 else FP32_PEAK_TFLOPS
    out = {
        "metric": "env-steps/sec (rollout+GAE+PPO update), 4096 envs, 16x16 mediumhard",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        # fp32 operands and results throughout; fc1's and the window GEMMs form their fp32 products from two f16
        # planes per operand (h3: three f16 MFMA products; error vs float64 no larger than hipBLASLt's fp32 GEMM,
        # tests/test_gpu_h3.py), exact to 2^-23 relative for values within 2^26 of each tensor's max |x|
        "dtype": "fp32",
        "dtype_note": ("fp32 operands/results; GEMM products as f16 two-plane (h3) splits with per-tensor power-of-two "
                       "scales: each value held to 2^-23 relative when within 2^26 of its tensor's scale reference "
                       "(smaller values to 2^-50 of it, absolute); the reference is max |x| for the weights and a "
                       "bound >= max |x| known before the producer runs for fc1's activations (dz: the loss's "
                       "gradient maxima through the heads' weights; a3: relu(b3 + sum over taps of Q's column maxima))"
                       ) if fc1 == "h3" else None,
        "data": "synthetic: procedurally generated mediumhard maps (numpy-PCG64-exact, seeds 777+i), "
                "random-init CNNActorCritic (torch seed 777), timed after the warm-up iterations",
        "config": {"workload": f"{args.difficulty} {args.size}x{args.size}, {N} envs/GPU x k_steps {T}, "
                               f"{args.epochs} epochs x {args.minibatches} minibatches of {B // args.minibatches}",
                   "num_envs_per_gpu": N, "k_steps": T, "global_batch": B * world,
                   "parallelism": f"dp{world}" if world > 1 else "single",
                   # the training state the number is measured at: the throughput depends on how many
                   # distinct frames / windows the policy's rollouts hold (distinct_frames_per_sample)
                   "state": f"iterations {args.warmup + 1}..{args.warmup + args.steps} of a run from random init "
                            f"(seed 777)"},
        # the number's data dependence: distinct observations per minibatch sample (1.0 = none repeat)
        "distinct_frames_per_sample": (round(agent.last_distinct_frac, 4)
                                       if agent.last_distinct_frac is not None else None),
        # dominant kernel of the timed loop by total HIP-event time (hand-written kernels and the
        # fc1 hipBLASLt GEMMs, which are timed the same way)
        "roofline": dict(roofline_of(dominant, kernels[dominant], fc1),
                         **({"note": "in the loop the weight gradient runs on a side stream beside conv3's "
                                     "backward segmented sums, so its event time includes that sharing; "
                                     "alone: roofline_x6_standalone"}
                            if dominant == "gemm_wgrad" and x6 and wgrad_side() else {})),
        # dominant hand-written kernel
        "roofline_handwritten": dict(roofline_of(handwritten, kernels[handwritten]),
                                     **gather_note(handwritten, kernels[handwritten])),
        # every GEMM family timed in the loop: the plane-form ones (h3 / x6) against the 16-bit MFMA peak with the
        # executed plane products, hipBLASLt's against the f32 MFMA peak
        "roofline_gemm": {k: roofline_of(k, v, fc1) for k, v in kernels.items() if "tflops" in v},
        # fc1's GEMM form: h3 = f16 two-plane (3 products, error below hipBLASLt's fp32 GEMM), x6 = bf16 three-plane
        "fc1_impl": fc1,
        # the env-step kernel inside the timed loop (absent when the rollout replays as a graph:
        # no per-kernel events inside it); the HBM-scale measurement is tiers.env_only_2M_envs
        "roofline_env_step": roofline_of("k_env_step", kernels["k_env_step"]) if "k_env_step" in kernels else None,
        # whole iteration, counting the fp32 products actually computed (GEMMs of conv3 / fc1 / heads on the
        # evaluated frames and windows), against the ceiling of the instructions that compute them: with the h3 form
        # every such GEMM runs 3 f16 MFMA products per fp32 product, so the ceiling is the dense f16 peak / 3; the
        # reference formulation's count is given for comparison (reference-equivalent rate = value x that)
        "roofline_loop": {"bound": "mfma", "achieved": round(loop_tflops, 2), "peak": loop_peak,
                          "unit": "TFLOP/s (fp32 products)", "frac": round(loop_tflops / loop_peak, 4),
                          "peak_basis": (f"dense 16-bit MFMA {BF16_PEAK_TFLOPS:.0f} / {PLANE_PRODUCTS[fc1]} plane "
                                         f"products per fp32 product ({fc1})") if x6 else "f32 MFMA",
                          "executed_flop_per_env_step": round(exec_flop_per_step),
                          "reference_flop_per_env_step": ref_flop_per_step,
                          "reference_equivalent_tflops": round(value / world * ref_flop_per_step / 1e12, 2)},
        "phases_ms": {"rollout": round(rollout_ms, 2), "update": round(update_ms, 2)},
        # conv2/conv3 evaluated once per distinct receptive-field window (merlin/windows.py)
        "windows_per_update": agent.last_num_windows,
        "rollout_graph": agent._graph is not None,
        # the acting layout the rollout ran (CNNActorCritic.rollout_pack)
        "rollout_acting": ("all-windows conv3 table" if agent.rollout_all_windows else "per-frame conv2 lookups"),
        "kernels": kernels,
    }
    if rank_spread is not None:
        out["ranks"] = rank_spread
    if x6 and agent.last_distinct_frac is not None:
        # the x6 GEMMs alone at the update's shape (distinct frames per minibatch)
        U = int(round(agent.last_distinct_frac * (B // args.minibatches)))
        out["roofline_x6_standalone"] = x6_standalone(torch, U, device, fc1)
    state["phase"] = "tiers"
    if world > 1:
        out["tiers"] = "run at n_gpus=1 only (their agents' updates would all-reduce on the world group)"
    elif not args.no_tiers:
        floors = floor_tier(agent)
        fused, single = env_only_tier(torch, MerlinVecEnv, N, T, args.difficulty, args.size, device)
        out["tiers"] = {"env_only_fused_T_steps_per_launch": round(fused, 1),
                        "env_only_one_step_per_launch": round(single, 1),
                        "rollout_only": round(B / (rollout_ms / 1e3), 1),
                        "env_only_2M_envs": env_large_tier(torch, MerlinVecEnv, args.difficulty, args.size, device),
                        "full_loop_per_gpu": round(value / world, 1),
                        # the same loop right after the timed region with the observation reuse switched
                        # off (median of 3 after a warm-up iteration per setting): the data-independent floor
                        "full_loop_floor": floors,
                        "hard_22": hard22_tier(device, N, T, args.epochs, args.minibatches),
                        "fomaml": fomaml_tier(device, args.difficulty)}
    state["phase"] = "cpu_baseline"
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out), flush=True)
    if dp.enabled:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
