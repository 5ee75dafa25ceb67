"""PPO training CLI -- drop-in for the reference's ppo/ppo_train.py (flags :19-41, loop :112-196).

    python ppo-2dgrid_amd/ppo_train.py --difficulty mediumhard --seed 777 --total_steps 10000
    python ppo-2dgrid_amd/ppo_train.py --difficulty mediumhard --num_envs 4096 --k_steps 256 ...
    torchrun --nproc-per-node 8 ppo-2dgrid_amd/ppo_train.py --num_envs 4096 --k_steps 256 ...

Same flags and defaults as the reference, plus:
  --num_envs N      parallel GPU envs per rank (default 1 = the reference's single env)
  --k_steps T       env steps per rollout; sets batch_size = num_envs * k_steps
  --size S          grid side override (default: scenario.yaml, 16)
  --stuck_penalty / --exploration_bonus [--bonus B]   reward-shaping flags (off by default)
  --config PATH     scenario YAML (default: the packaged copy of src/config/scenario.yaml)
Outputs keep the reference's layout: checkpoints/<env_id>_<WxH>_<difficulty>_<ts>/seed_<s>/
{best_model, ppo_model_<k>k, ppo_model_final}.pth (CNNActorCritic state_dicts with the
reference's keys) and tb_logs/... scalars (TensorBoard when installed, else scalars.jsonl).
Env seeding: env i of rank r is reset once with seed + r*num_envs + i (the reference's
training env is unseeded); eval episodes use seed+999+ep like :48.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import datetime

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merlin import PPO, ScenarioCreator  # noqa: E402
from merlin.distributed import DataParallel  # noqa: E402
from merlin.evaluation import evaluate_policy  # noqa: E402
from merlin.metrics.ppo_metrics import compute_episode_stats  # noqa: E402
from merlin.scenario_creator import DEFAULT_CONFIG  # noqa: E402
from merlin.utils.utils import get_device, set_seed  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--device", type=str, default="auto")
    p.add_argument("--lr", type=float, default=3e-4)
    p.add_argument("--gamma", type=float, default=0.99)
    p.add_argument("--lam", type=float, default=0.95)
    p.add_argument("--clip_eps", type=float, default=0.2)
    p.add_argument("--update_epochs", type=int, default=10)
    p.add_argument("--batch_size", type=int, default=2048)
    p.add_argument("--minibatch_size", type=int, default=256)
    p.add_argument("--vf_coef", type=float, default=0.5)
    p.add_argument("--ent_coef", type=float, default=0.05)
    p.add_argument("--total_steps", type=int, default=300_000)
    p.add_argument("--save_interval", type=int, default=100_000)
    p.add_argument("--eval_episodes", type=int, default=3)
    p.add_argument("--log_dir", type=str, default="logs")
    p.add_argument("--ckpt_dir", type=str, default="checkpoints")
    p.add_argument("--visual_eval", action="store_true")
    p.add_argument("--print_interval", type=int, default=2048)
    p.add_argument("--difficulty", type=str, default="easy",
                   choices=["easy", "medium", "mediumhard", "hard", "hardest"])
    p.add_argument("--seed", type=int, default=123)
    p.add_argument("--group_timestamp", type=str, default=None)
    # MERLIN-AMD additions
    p.add_argument("--num_envs", type=int, default=1)
    p.add_argument("--k_steps", type=int, default=None)
    p.add_argument("--size", type=int, default=None)
    p.add_argument("--stuck_penalty", action="store_true")
    p.add_argument("--exploration_bonus", action="store_true")
    p.add_argument("--bonus", type=float, default=0.01)
    p.add_argument("--config", type=str, default=DEFAULT_CONFIG)
    return p.parse_args(argv)


class ScalarLog:
    """TensorBoard SummaryWriter when available, else a JSONL file with the same tags."""

    def __init__(self, path: str):
        os.makedirs(path, exist_ok=True)
        try:
            from torch.utils.tensorboard import SummaryWriter

            self.tb, self.f = SummaryWriter(log_dir=path), None
        except Exception:
            self.tb, self.f = None, open(os.path.join(path, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, step):
        if self.tb is not None:
            self.tb.add_scalar(tag, value, step)
        else:
            self.f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")

    def add_histogram(self, tag, values, step):
        values = np.asarray(values, dtype=np.float64)
        if self.tb is not None:
            self.tb.add_histogram(tag, values, step)
        else:
            counts, edges = np.histogram(values, bins=min(30, max(1, values.size)))
            self.f.write(json.dumps({"tag": tag, "histogram": {"counts": counts.tolist(), "edges": edges.tolist()},
                                     "step": int(step)}) + "\n")

    def add_reward_vs_steps(self, tag, lengths, returns, step):
        """The reference's scatter figure (ppo/ppo_train.py:186-190): a matplotlib figure in
        TensorBoard, the raw points in the JSONL stand-in."""
        if self.tb is not None:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt

            fig = plt.figure()
            plt.scatter(lengths, returns, c="green")
            self.tb.add_figure(tag, fig, step)
            plt.close(fig)
        else:
            self.f.write(json.dumps({"tag": tag, "points": [[float(a), float(b)] for a, b in zip(lengths, returns)],
                                     "step": int(step)}) + "\n")

    def close(self):
        if self.tb is not None:
            self.tb.close()
        else:
            self.f.close()


def train_minigrid(args):
    set_seed(args.seed)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = get_device(args.device)
    dp = DataParallel.init_from_env(device=device)
    if device.type != "cuda":
        raise SystemExit("merlin trains on a GPU (HIP) device; none is visible")

    sc = ScenarioCreator(args.config)
    flags = dict(stuck_penalty=args.stuck_penalty, exploration_bonus=args.exploration_bonus, bonus=args.bonus)
    size_kw = {} if args.size is None else {"size": args.size}
    batch = args.num_envs * args.k_steps if args.k_steps else args.batch_size
    if args.num_envs > 1:
        env = sc.create_vec_env(args.difficulty, args.num_envs, seed=args.seed, device=device,
                                env_offset=rank * args.num_envs, **size_kw, **flags)
    else:
        # rank r's single env is global env r: seed + r, and its action draws are keyed by r
        env = sc.create_env(args.difficulty, seed=args.seed, device=device, env_offset=rank, **size_kw, **flags)
        env.vec.set_base_seed(args.seed)  # create_env ignores its seed, like the reference's
    agent = PPO(env, lr=args.lr, gamma=args.gamma, lam=args.lam, clip_eps=args.clip_eps,
                update_epochs=args.update_epochs, batch_size=batch, minibatch_size=args.minibatch_size,
                vf_coef=args.vf_coef, ent_coef=args.ent_coef, device=device, dp=dp)

    env_id = sc.get_env_id(args.difficulty)
    size = args.size or int(sc.get_env_size_str(args.difficulty).split("x")[0])
    grid_size_str = f"{size}x{size}"
    timestamp = args.group_timestamp or datetime.now().strftime("%Y%m%d_%H%M%S")
    experiment_name = f"{env_id}_{grid_size_str}_{args.difficulty}_{timestamp}"
    ckpt_subdir = os.path.join(args.ckpt_dir, experiment_name, f"seed_{args.seed}")
    tb_dir = os.path.join("tb_logs", experiment_name, f"seed_{args.seed}")
    lead = rank == 0
    if lead:
        os.makedirs(ckpt_subdir, exist_ok=True)
        writer = ScalarLog(tb_dir)
    best_model_path = os.path.join(ckpt_subdir, "best_model.pth")

    step_count, next_save = 0, args.save_interval
    start_time = time.time()
    best_reward = -float("inf")
    steps_per_iter = agent.batch_size * dp.world
    while step_count < args.total_steps:
        t0 = time.time()
        last_value = agent.collect_rollouts()
        update_stats = agent.update(last_value)
        step_count += steps_per_iter
        sps = steps_per_iter / (time.time() - t0)
        if not lead:
            continue
        eval_rewards, eval_steps = evaluate_policy(agent.ac, args.difficulty, episodes=args.eval_episodes,
                                                   seed=args.seed + 999, size=size, device=device, **flags)
        avg_r, avg_s = float(np.mean(eval_rewards)), float(np.mean(eval_steps))
        if avg_r > best_reward:
            best_reward = avg_r
            torch.save(agent.ac.state_dict(), best_model_path)
            print(f"[*] New best PPO model saved! Reward: {best_reward:.3f} -> {best_model_path}")
        if step_count >= next_save or step_count >= args.total_steps:
            torch.save(agent.ac.state_dict(), os.path.join(ckpt_subdir, f"ppo_model_{int(step_count / 1000)}k.pth"))
            next_save += args.save_interval
        writer.add_scalar("reward/avg_eval_reward", avg_r, step_count)
        for tag, key in (("loss/policy_loss", "pi_loss"), ("loss/value_loss", "v_loss"), ("loss/entropy", "entropy"),
                         ("diagnostics/kl", "kl"), ("diagnostics/clipfrac", "clipfrac"),
                         ("diagnostics/gradnorm", "gradnorm")):
            writer.add_scalar(tag, update_stats[key], step_count)
        writer.add_scalar("perf/env_steps_per_sec", sps, step_count)
        if agent.episode_returns:
            st = compute_episode_stats(agent.episode_returns[-10:], agent.episode_lengths[-10:])
            writer.add_scalar("stats/episode_return_mean", st["episode_return_mean"], step_count)
            writer.add_scalar("stats/episode_length_mean", st["episode_length_mean"], step_count)
        if step_count % args.print_interval == 0 or step_count >= args.total_steps or steps_per_iter > args.print_interval:
            elapsed_min = (time.time() - start_time) / 60
            total_loss = update_stats["pi_loss"] + update_stats["v_loss"]
            print(f"[{step_count:>7}] R: {avg_r:.3f} | L: {total_loss:.4f} | pi: {update_stats['pi_loss']:.4f} | "
                  f"V: {update_stats['v_loss']:.4f} | Ent: {update_stats['entropy']:.4f} | "
                  f"KL: {update_stats['kl']:.6f} | Steps: {avg_s:.1f} | T: {elapsed_min:.2f}m | {sps:,.0f} steps/s",
                  flush=True)
            if len(agent.episode_returns) >= 10:  # ppo/ppo_train.py:184-190
                writer.add_histogram("hist/episode_rewards", agent.episode_returns[-50:], step_count)
                writer.add_histogram("hist/episode_lengths", agent.episode_lengths[-50:], step_count)
                writer.add_reward_vs_steps("fig/reward_vs_steps", agent.episode_lengths[-50:],
                                           agent.episode_returns[-50:], step_count)
    if lead:
        torch.save(agent.ac.state_dict(), os.path.join(ckpt_subdir, "ppo_model_final.pth"))
        writer.close()
    return agent


if __name__ == "__main__":
    train_minigrid(parse_args())
