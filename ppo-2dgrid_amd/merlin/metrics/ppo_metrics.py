"""PPO update / episode statistics (src/metrics/ppo_metrics.py:7-57 of the reference)."""
from __future__ import annotations

from typing import Dict, List

_KEYS = ("pi_loss", "v_loss", "entropy", "kl", "clipfrac", "gradnorm")


def aggregate_ppo_update_metrics(total_pi: float, total_v: float, total_ent: float, total_kl: float,
                                 total_clip: float, total_gnorm: float, nbatches: int) -> Dict[str, float]:
    """Mean of the per-minibatch totals; zeros when no minibatch ran (ppo_metrics.py:7-40)."""
    if nbatches == 0:
        return {k: 0.0 for k in _KEYS}
    totals = (total_pi, total_v, total_ent, total_kl, total_clip, total_gnorm)
    return {k: float(v) / nbatches for k, v in zip(_KEYS, totals)}


def compute_episode_stats(episode_returns: List[float], episode_lengths: List[int]) -> Dict[str, float]:
    """(ppo_metrics.py:43-57)"""
    if len(episode_returns) == 0:
        return {"episode_return_mean": 0.0, "episode_length_mean": 0.0}
    return {
        "episode_return_mean": sum(episode_returns) / len(episode_returns),
        "episode_length_mean": sum(episode_lengths) / len(episode_lengths),
    }
