"""Functional CNNActorCritic with one weight set per group (task), batched over groups.

FOMAML (src/fomaml.py:158-223) adapts a separate copy of the policy per task.  Instead of
looping over tasks, the per-task copies live as stacked tensors [G, *shape] (keys of
CNNActorCritic.state_dict) and one forward evaluates every task's samples with its own
weights: each convolution is an unfold + batched matmul over groups, each Linear a batched
matmul.  Autograd through it gives every task's gradient at once, since tasks share no
parameters.  Inputs are frames already divided by 255 ([G, B, 3, 56, 56], e.g. from
merlin_obs_expand_f32 with scale 1/255).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_CONVS = ((0, 4), (2, 2), (4, 1))  # (network index, stride) -- actor_critic.py:9-14


def stack_params(model: torch.nn.Module, groups: int) -> dict:
    """[G, *shape] copies of every parameter (detached, grad-enabled leaves)."""
    return {k: v.detach().unsqueeze(0).repeat(groups, *([1] * v.dim())).requires_grad_(True)
            for k, v in model.named_parameters()}


def _conv(x, w, b, stride, G):
    # x [G*B, Cin, H, W]; w [G, Cout, Cin, k, k]; b [G, Cout] -> relu(conv) [G*B, Cout, Ho, Wo]
    GB, cin, H, W = x.shape
    B = GB // G
    cout, k = w.shape[1], w.shape[-1]
    ho, wo = (H - k) // stride + 1, (W - k) // stride + 1
    cols = F.unfold(x, kernel_size=k, stride=stride).view(G, B, cin * k * k, ho * wo)
    y = torch.einsum("gok,gbkp->gbop", w.reshape(G, cout, cin * k * k), cols) + b[:, None, :, None]
    return torch.relu(y).reshape(GB, cout, ho, wo)


def _tower(params, prefix, x, G):
    for idx, stride in _CONVS:
        x = _conv(x, params[f"{prefix}.network.{idx}.weight"], params[f"{prefix}.network.{idx}.bias"], stride, G)
    return x.reshape(G, x.shape[0] // G, -1)  # Flatten: (c, y, x) order, as nn.Flatten


def _mlp_head(params, prefix, h):
    w0, b0 = params[f"{prefix}.0.weight"], params[f"{prefix}.0.bias"]
    w2, b2 = params[f"{prefix}.2.weight"], params[f"{prefix}.2.bias"]
    h = torch.relu(torch.einsum("gbk,gjk->gbj", h, w0) + b0[:, None, :])
    return torch.einsum("gbj,gaj->gba", h, w2) + b2[:, None, :]


def forward(params: dict, frames: torch.Tensor):
    """frames [G, B, 3, H, W] (/255) -> logits [G, B, A], values [G, B]."""
    G, B = frames.shape[:2]
    x = frames.reshape(G * B, *frames.shape[2:])
    logits = _mlp_head(params, "actor", _tower(params, "actor_extractor", x, G))
    value = _mlp_head(params, "critic", _tower(params, "critic_extractor", x, G)).squeeze(-1)
    return logits, value


def _categorical(logits):
    logp = logits - logits.logsumexp(dim=-1, keepdim=True)
    return logp, F.softmax(logp, dim=-1)


def act(params, frames, deterministic=False):
    """CNNActorCritic.act per group: (action [G, B], logp [G, B], value [G, B])."""
    logits, value = forward(params, frames)
    logp_all, probs = _categorical(logits)
    if deterministic:
        a = logits.argmax(dim=-1)
    else:
        a = torch.multinomial(probs.reshape(-1, probs.shape[-1]), 1, True).reshape(probs.shape[:-1])
    return a, logp_all.gather(-1, a.unsqueeze(-1)).squeeze(-1), value


def evaluate(params, frames, actions):
    """CNNActorCritic.evaluate per group: (logp, entropy, value), each [G, B]."""
    logits, value = forward(params, frames)
    logp_all, probs = _categorical(logits)
    logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
    ent = -(torch.clamp(logp_all, min=torch.finfo(logp_all.dtype).min) * probs).sum(-1)
    return logp, ent, value
