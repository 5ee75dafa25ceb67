"""Checkpoint sweep CLI -- drop-in for the reference's src/sweep_checkpoints.py (flags :11-17).

    python ppo-2dgrid_amd/sweep_checkpoints.py --model_dir checkpoints/<exp>/seed_777 --tasks 100

Every *.pth in --model_dir (current or legacy feature_extractor.conv layout) is evaluated
deterministically on the fixed seeds 200000 .. 200000+tasks-1, all episodes of a checkpoint at once
on the GPU envs (merlin.evaluation.sweep_checkpoints), and ranked by mean reward.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from merlin.evaluation import sweep_checkpoints  # noqa: E402
from merlin.scenario_creator import DEFAULT_CONFIG, ScenarioCreator  # noqa: E402
from merlin.utils.utils import get_device  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--difficulty", type=str, default="mediumhard")
    p.add_argument("--model_dir", type=str, required=True)
    p.add_argument("--tasks", type=int, default=50)
    p.add_argument("--config", type=str, default=DEFAULT_CONFIG)
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    device = get_device("auto")
    sc = ScenarioCreator(args.config)
    size = int(sc.get_env_size_str(args.difficulty).split("x")[0])
    print(f"[*] Fixed Evaluation Tasks: {args.tasks}")
    results = sweep_checkpoints(args.model_dir, args.difficulty, args.tasks, size=size, device=device)
    if not results:
        print(f"[*] No .pth files found in {args.model_dir}")
        return results
    print("=" * 60)
    print(f"{'RANK':<5} | {'CHECKPOINT':<25} | {'REWARD':<8} | {'STEPS'}")
    print("=" * 60)
    for rank, (mp, r, s) in enumerate(results, 1):
        print(f"#{rank:<4} | {os.path.basename(mp):<25} | {r:<8.3f} | {s:.1f}")
    print("=" * 60)
    return results


if __name__ == "__main__":
    main()
