"""Identical observations in a minibatch share one tower evaluation.

A MiniGrid observation is a 7x7 view of 5 tile classes, and a rollout revisits the same
views often (measured on the bench rollout, 4096 mediumhard envs x 256 random-action
steps: 27 % of the 1,048,576 frames are distinct overall, 61 % inside a 131,072-frame
minibatch; hard 22x22: 7 % / 19 %).  The CNN towers are a deterministic function of the
observation, so a minibatch's logits/values are tower(unique frames)[inverse]: the forward
runs once per distinct frame and autograd's index_select backward sums the per-sample
gradients of equal frames before the tower backward.  Same function and gradient as
evaluating every sample (src/ppo.py:136-156), fp32 sums regrouped; nothing is cached
across optimizer steps (the towers run with the current weights for every minibatch).

Frame identity: a 64-bit hash of the 32-byte codes picks the groups, and every frame is
then compared word for word with its group's representative, so a hash collision can
never merge two different observations (the update falls back to per-sample towers).
"""
from __future__ import annotations

import torch

# odd 64-bit multipliers (splitmix64 constants and their relatives), one per code word
_MULT = (0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 0xD6E8FEB86659FD93,
         0xA0761D6478BD642F, 0xE7037ED1A0B428DB, 0x8EBC6AF09C88C6E3, 0x589965CC75374CC3)


def _signed(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


def hash_codes(codes: torch.Tensor) -> torch.Tensor:
    """int32 [B, 8] -> int64 [B] (wrapping 64-bit arithmetic)."""
    w = codes.to(torch.int64) & 0xFFFFFFFF
    h = torch.zeros(codes.shape[0], dtype=torch.int64, device=codes.device)
    for k in range(codes.shape[1]):
        h = (h ^ w[:, k]) * _signed(_MULT[k])
        h = h ^ ((h >> 29) & ((1 << 35) - 1))  # logical shift of the signed value
    return h


class FrameGroups:
    """Group ids of a rollout's frames, computed once per update.

    uid[i] in [0, U) for frame i; rep[u] = one frame index of group u.  ``ok`` is False
    when the hash grouping would merge different observations (then callers skip dedup).
    """

    def __init__(self, codes: torch.Tensor):
        h = hash_codes(codes)
        uniq, uid = torch.unique(h, return_inverse=True)
        U = uniq.numel()
        rep = torch.empty(U, dtype=torch.int64, device=codes.device)
        rep.scatter_(0, uid, torch.arange(codes.shape[0], device=codes.device))
        self.ok = bool(torch.equal(codes[rep[uid]], codes))
        self.uid, self.rep, self.num_groups = uid, rep, U

    def minibatch(self, mb_idx: torch.Tensor):
        """(rep_idx [u], inv [n]): the minibatch's distinct frames (as frame indices) and, per
        sample, its position in rep_idx."""
        u, inv = torch.unique(self.uid[mb_idx], return_inverse=True)
        return self.rep[u], inv
