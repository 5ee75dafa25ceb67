"""RL utilities mirroring src/utils/utils_rl.py of the reference.

``layer_init``            orthogonal init (utils_rl.py:6-9), identical calls so that a
                          model built under the same torch seed gets the same weights.
``compute_gae_standard``  stateless GAE (utils_rl.py:11-29, used by FOMAML) computed by
                          the HIP kernel (merlin_gae) on device tensors.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native as nat


def layer_init(layer, std=np.sqrt(2), bias_const=0.0):
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


def compute_gae_standard(rewards, values, dones, last_value, gamma=0.99, lam=0.95, device="cuda"):
    """GAE of one trajectory ([T]) or T x N rollouts ([T, N]); returns (adv, returns).

    numpy inputs give numpy float32 outputs (the reference's contract); tensors stay
    on their device.  The computation itself always runs in the HIP kernel."""
    as_numpy = isinstance(rewards, np.ndarray)
    dev = torch.device(device) if as_numpy else rewards.device

    def to_t(x):
        return torch.as_tensor(np.asarray(x, dtype=np.float32) if as_numpy else x, dtype=torch.float32,
                               device=dev).contiguous()

    r, v, d = to_t(rewards), to_t(values), to_t(dones)
    n = r.numel() // r.shape[0]
    lv = torch.as_tensor(last_value, dtype=torch.float32, device=dev).reshape(-1)
    if lv.numel() == 1 and n > 1:
        lv = lv.expand(n).contiguous()
    adv, ret = nat.gae(r, v, d, lv, gamma, lam)
    if as_numpy:
        return adv.cpu().numpy(), ret.cpu().numpy()
    return adv, ret
