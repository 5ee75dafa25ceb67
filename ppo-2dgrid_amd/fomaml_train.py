"""FOMAML training CLI -- drop-in for the reference's fomaml/fomaml_train.py (flags :16-35).

    python ppo-2dgrid_amd/fomaml_train.py --difficulty mediumhard --tasks_per_batch 32 --k_steps 256

Tasks per meta-iteration are sampled like the reference (:101): np.random.choice(range(100000),
tasks_per_batch, replace=False) from the seeded global numpy RNG; all tasks run batched on the
GPU (merlin.fomaml).  Outputs follow the reference (:48-51, :128-174):
checkpoints/<env_id>_<WxH>_<difficulty>_FOMAML_<ts>/seed_<s>/ holds best_model.pth (saved whenever the
meta-iteration's query reward beats the best so far), fomaml_iter_<k>.pth and training_curves.png every
100 iterations (``--save_every``, an added flag, default the reference's 100), the figure drawn on
matplotlib's Agg backend (skipped with a note when matplotlib is absent).  The per-10-iteration line
carries the reference's fields (:136).  --render_live / --plot_curves are accepted and ignored: they
open interactive windows, and the GPU nodes have no display.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from datetime import datetime

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merlin import ScenarioCreator  # noqa: E402
from merlin.fomaml import FOMAML  # noqa: E402
from merlin.utils.utils import get_device, set_seed  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Train FOMAML on MiniGrid")
    p.add_argument("--difficulty", type=str, default="medium", choices=["easy", "medium", "mediumhard", "hard", "hardest"])
    p.add_argument("--iterations", type=int, default=2000, help="Total meta-training iterations")
    p.add_argument("--tasks_per_batch", type=int, default=8, help="Number of tasks (maps) to sample per meta-update")
    p.add_argument("--k_steps", type=int, default=256, help="Trajectory length for Support and Query sets")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--device", type=str, default="auto")
    p.add_argument("--render_live", action="store_true", default=False)
    p.add_argument("--plot_curves", action="store_true", default=False)
    p.add_argument("--save_every", type=int, default=100,
                   help="iterations between fomaml_iter_<k>.pth / training_curves.png (reference: 100)")
    return p.parse_args(argv)


def save_training_curves(history, path):
    """The reference's two-panel figure (:142-157): avg query reward and steps per iteration.
    Returns False (and writes nothing) when matplotlib is not importable."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return False
    fig, ax = plt.subplots(2, 1, figsize=(10, 8))
    ax[0].plot(history["iter"], history["rew"], color="green", label="Avg Reward")
    ax[0].set_title("Meta-Test Reward")
    ax[0].set_ylabel("Reward (0-1)")
    ax[0].grid(True, alpha=0.3)
    ax[1].plot(history["iter"], history["steps"], color="blue", label="Steps to Goal")
    ax[1].set_title("Navigation Efficiency")
    ax[1].set_ylabel("Steps")
    ax[1].set_xlabel("Iterations")
    ax[1].grid(True, alpha=0.3)
    fig.savefig(path)
    plt.close(fig)
    return True


def train_fomaml(args):
    set_seed(args.seed)
    device = get_device(args.device)
    sc = ScenarioCreator()
    env_id = sc.get_env_id(args.difficulty)
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    project_name = f"{env_id}_{sc.get_env_size_str(args.difficulty)}_{args.difficulty}_FOMAML_{ts}"
    ckpt_dir = os.path.join("checkpoints", project_name, f"seed_{args.seed}")
    os.makedirs(ckpt_dir, exist_ok=True)
    fomaml = FOMAML(sc, lr_inner=0.01, lr_outer=3e-4, difficulty=args.difficulty, device=device)
    print("==================================================")
    print("[FOMAML] Starting Meta-Training")
    print(f" Project      : {project_name}")
    print(f" Difficulty   : {args.difficulty}")
    print(f" Env ID       : {env_id}")
    print(f" Seed         : {args.seed}")
    print(f" Saving to    : {ckpt_dir}")
    print(f" Live Map     : {'ON' if args.render_live else 'OFF'}")
    print(f" Live Curves  : {'ON' if args.plot_curves else 'OFF'}")
    print("==================================================", flush=True)
    best = -float("inf")
    history = {"iter": [], "loss": [], "rew": [], "steps": []}
    t0 = time.time()
    for itr in range(1, args.iterations + 1):
        seeds = [int(s) for s in np.random.choice(range(100000), size=args.tasks_per_batch, replace=False)]
        loss, rew, steps, stats = fomaml.meta_train_step(seeds, k_support=args.k_steps, k_query=args.k_steps)
        history["iter"].append(itr)
        history["loss"].append(loss)
        history["rew"].append(rew)
        history["steps"].append(steps)
        if rew > best:
            best = rew
            torch.save(fomaml.meta_policy.state_dict(), os.path.join(ckpt_dir, "best_model.pth"))
            print(f"[*] New Best Model Saved (Rew: {best:.4f})")
        if itr % 10 == 0:
            elapsed = (time.time() - t0) / 60
            print(f"Iter {itr:>4} | R: {rew:.3f} | L: {loss:.4f} | pi: {stats['pi_loss']:.4f} | "
                  f"V: {stats['v_loss']:.4f} | Ent: {stats['entropy']:.4f} | KL: {stats['kl']:.6f} | "
                  f"Steps: {steps:.1f} | Best: {best:.4f} | T: {elapsed:.1f}m", flush=True)
        if itr % args.save_every == 0:
            torch.save(fomaml.meta_policy.state_dict(), os.path.join(ckpt_dir, f"fomaml_iter_{itr}.pth"))
            plot_path = os.path.join(ckpt_dir, "training_curves.png")
            if save_training_curves(history, plot_path):
                print(f"[*] Saved training curves to: {plot_path}", flush=True)
            else:
                print("[!] matplotlib is not importable: training_curves.png skipped", flush=True)
    return fomaml


if __name__ == "__main__":
    train_fomaml(parse_args())
