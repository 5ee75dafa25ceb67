"""Seeding and device selection (src/utils/utils.py:5-46 of the reference)."""
from __future__ import annotations

import random

import numpy as np
import torch


def set_seed(seed, deterministic: bool = True):
    """random / numpy / torch seeding (utils.py:5-13).  Like the reference this does
    not seed the env RNG; envs are seeded through MerlinVecEnv(seed=...)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
        torch.backends.cudnn.deterministic = deterministic
        torch.backends.cudnn.benchmark = not deterministic


def get_device(device_str="cpu"):
    """"cpu" / "cuda" / "cuda:k" / "auto" (utils.py:15-46).

    Deviation: "auto" without a GPU returns CPU instead of MPS (the reference picks
    MPS, which does not exist on Linux); the HIP paths then refuse to run."""
    if device_str == "auto":
        if torch.cuda.is_available():
            print(f"Device set to: {torch.cuda.get_device_name(0)} (cuda:0)")
            return torch.device("cuda:0")
        print("Device set to: CPU (no GPU visible)")
        return torch.device("cpu")
    if device_str.startswith("cuda"):
        if torch.cuda.is_available():
            print(f"Device set to: {torch.cuda.get_device_name(0)} ({device_str})")
            return torch.device(device_str)
        print("[WARNING] CUDA requested but not available → using CPU")
        return torch.device("cpu")
    if device_str == "cpu":
        print("Device set to: CPU")
        return torch.device("cpu")
    print("[WARNING] Unknown device flag, defaulting to CPU")
    return torch.device("cpu")
