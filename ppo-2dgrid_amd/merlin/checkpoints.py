"""Checkpoint interop with the reference's ``.pth`` files.

``CNNActorCritic.state_dict()`` keys are the reference's (src/actor_critic.py), so current
checkpoints load unchanged.  Older reference checkpoints kept ONE shared conv stack under
``feature_extractor.conv.*``; the reference's loaders (src/sweep_checkpoints.py:31-47,
fomaml/fomaml_visualization.py:110-122) copy it into both towers and load non-strictly.
``remap_legacy_state_dict`` / ``load_policy`` do the same.  Files are read with
``torch.load(weights_only=True)`` (nothing in them is executed).
"""
from __future__ import annotations

import torch

from .actor_critic import CNNActorCritic

LEGACY_PREFIX = "feature_extractor.conv"


def is_legacy(state_dict) -> bool:
    return any("feature_extractor" in k for k in state_dict)


def remap_legacy_state_dict(state_dict) -> dict:
    """feature_extractor.conv.* -> actor_extractor.network.* and critic_extractor.network.* (cloned);
    other keys unchanged (src/sweep_checkpoints.py:35-45)."""
    out = {}
    for k, v in state_dict.items():
        if LEGACY_PREFIX in k:
            out[k.replace(LEGACY_PREFIX, "actor_extractor.network")] = v.clone()
            out[k.replace(LEGACY_PREFIX, "critic_extractor.network")] = v.clone()
        else:
            out[k] = v
    return out


def load_policy(path: str, device="cuda", obs_shape=(56, 56, 3), act_dim: int = 3) -> CNNActorCritic:
    """A CNNActorCritic with the weights of a reference .pth (current or legacy layout), in eval mode
    (src/sweep_checkpoints.py:19-50)."""
    policy = CNNActorCritic(obs_shape, act_dim).to(device)
    sd = torch.load(path, map_location=device, weights_only=True)
    if is_legacy(sd):
        print(f"[*] Warning: Legacy model architecture detected in {path}. Mapping weights...")
        policy.load_state_dict(remap_legacy_state_dict(sd), strict=False)
    else:
        policy.load_state_dict(sd)
    policy.eval()
    return policy
