"""FOMAML training CLI -- drop-in for the reference's fomaml/fomaml_train.py (flags :16-35).

    python ppo-2dgrid_amd/fomaml_train.py --difficulty mediumhard --tasks_per_batch 32 --k_steps 256

Tasks per meta-iteration are sampled like the reference (:101): np.random.choice(range(100000),
tasks_per_batch, replace=False) from the seeded global numpy RNG; all tasks run batched on the
GPU (merlin.fomaml).  Checkpoints: checkpoints/<env_id>_<WxH>_<difficulty>_FOMAML_<ts>/seed_<s>/.
--render_live / --plot_curves are accepted and ignored (no display on the GPU nodes).
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
    p.add_argument("--iterations", type=int, default=2000)
    p.add_argument("--tasks_per_batch", type=int, default=8)
    p.add_argument("--k_steps", type=int, default=256)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--device", type=str, default="auto")
    p.add_argument("--render_live", action="store_true", default=False)
    p.add_argument("--plot_curves", action="store_true", default=False)
    p.add_argument("--save_every", type=int, default=100)
    return p.parse_args(argv)


def train_fomaml(args):
    set_seed(args.seed)
    device = get_device(args.device)
    sc = ScenarioCreator()
    env_id = sc.get_env_id(args.difficulty)
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    ckpt_dir = os.path.join("checkpoints", f"{env_id}_{sc.get_env_size_str(args.difficulty)}_{args.difficulty}_FOMAML_{ts}",
                            f"seed_{args.seed}")
    os.makedirs(ckpt_dir, exist_ok=True)
    fomaml = FOMAML(sc, lr_inner=0.01, lr_outer=3e-4, difficulty=args.difficulty, device=device)
    best = -float("inf")
    t0 = time.time()
    for itr in range(1, args.iterations + 1):
        seeds = np.random.choice(range(100000), args.tasks_per_batch, replace=False)
        loss, rew, steps, stats = fomaml.meta_train_step(seeds, k_support=args.k_steps, k_query=args.k_steps)
        if rew > best:
            best = rew
            torch.save(fomaml.meta_policy.state_dict(), os.path.join(ckpt_dir, "fomaml_best.pth"))
        if itr % args.save_every == 0:
            torch.save(fomaml.meta_policy.state_dict(), os.path.join(ckpt_dir, f"fomaml_iter_{itr}.pth"))
        if itr % 10 == 0 or itr == 1:
            print(f"Iter {itr:4d} | Loss: {loss:.4f} | Reward: {rew:.3f} | Steps: {steps:.1f} | "
                  f"KL: {stats['kl']:.5f} | T: {(time.time() - t0) / 60:.2f}m", flush=True)
    torch.save(fomaml.meta_policy.state_dict(), os.path.join(ckpt_dir, "fomaml_final.pth"))
    return fomaml


if __name__ == "__main__":
    train_fomaml(parse_args())
