"""Actor-critic networks: the model-side drop-in surface (src/actor_critic.py).

Frozen contract with the reference:
  * ``CNNActorCritic(obs_shape=(H, W, C), act_dim, hidden_dim=512)`` with separate
    actor / critic towers conv(C->32,k8,s4) -> conv(32->64,k4,s2) -> conv(64->64,k3,s1)
    -> flatten -> Linear(hidden) -> ReLU -> Linear(act_dim | 1); state_dict keys
    ``{actor,critic}_extractor.network.{0,2,4}.*`` and ``{actor,critic}.{0,2}.*``,
    so reference ``.pth`` checkpoints load unchanged (actor_critic.py:6-41);
  * modules are created and initialised in the reference's order, so the same
    torch seed gives the same weights (layer_init, utils_rl.py:6-9);
  * ``act(obs, deterministic) -> (action, logp, value)`` and
    ``evaluate(obs, actions) -> (logp, entropy, value)`` (actor_critic.py:48-64),
    obs as float [B, H, W, C] in 0..255 (permuted like ``_format_obs``) or [B, C, H, W].

MERLIN-AMD addition: ``prescaled=True`` tells the towers that the input is already
divided by 255 (the HIP observation expansion folds the /255 of
CNNFeatureExtractor.forward, actor_critic.py:20-21, into its store), so the rollout
and update never materialise an extra scaled copy of the observation batch.
The categorical head is computed directly with log_softmax instead of building a
torch.distributions.Categorical per call (same formulas: log-prob of the
normalised logits, entropy = -sum p*log p).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .utils.utils_rl import layer_init

# (out_channels, kernel, stride) of the three convs -- actor_critic.py:9-14
_CONV_SPEC = ((32, 8, 4), (64, 4, 2), (64, 3, 1))


class CNNFeatureExtractor(nn.Module):
    def __init__(self, channels, height, width):
        super().__init__()
        layers = []
        cin = channels
        for cout, k, s in _CONV_SPEC:
            layers += [layer_init(nn.Conv2d(cin, cout, kernel_size=k, stride=s)), nn.ReLU()]
            cin = cout
        layers.append(nn.Flatten())
        self.network = nn.Sequential(*layers)
        with torch.no_grad():
            self.output_dim = self.network(torch.zeros(1, channels, height, width)).shape[1]

    def forward(self, x, prescaled: bool = False):
        return self.network(x if prescaled else x / 255.0)


def _head(in_dim: int, hidden: int, out_dim: int, out_std: float, act=nn.ReLU) -> nn.Sequential:
    return nn.Sequential(layer_init(nn.Linear(in_dim, hidden)), act(),
                         layer_init(nn.Linear(hidden, out_dim), std=out_std))


def _categorical(logits: torch.Tensor):
    """(normalised log-probs, probs) of Categorical(logits=...)."""
    logp = logits - logits.logsumexp(dim=-1, keepdim=True)
    return logp, F.softmax(logp, dim=-1)


def _sample_or_argmax(logits: torch.Tensor, logp_all: torch.Tensor, probs: torch.Tensor, deterministic: bool):
    if deterministic:
        return torch.argmax(logits, dim=1)
    return torch.multinomial(probs.reshape(-1, probs.shape[-1]), 1, True).reshape(probs.shape[:-1])


def _entropy(logp_all: torch.Tensor, probs: torch.Tensor) -> torch.Tensor:
    lp = torch.clamp(logp_all, min=torch.finfo(logp_all.dtype).min)
    return -(lp * probs).sum(-1)


class CNNActorCritic(nn.Module):
    def __init__(self, obs_shape, act_dim, hidden_dim=512):
        super().__init__()
        h, w, c = obs_shape
        self.actor_extractor = CNNFeatureExtractor(c, h, w)
        self.critic_extractor = CNNFeatureExtractor(c, h, w)
        self.actor = _head(self.actor_extractor.output_dim, hidden_dim, act_dim, 0.01)
        self.critic = _head(self.critic_extractor.output_dim, hidden_dim, 1, 1.0)

    def _format_obs(self, x):
        # NHWC observations (the gym frame layout) -> NCHW for the convs
        if x.ndim == 4 and x.shape[-1] == 3:
            return x.permute(0, 3, 1, 2).float()
        return x.float()

    def _forward(self, obs, prescaled: bool):
        obs = self._format_obs(obs)
        logits = self.actor(self.actor_extractor(obs, prescaled=prescaled))
        value = self.critic(self.critic_extractor(obs, prescaled=prescaled)).squeeze(-1)
        return logits, value

    def act(self, obs, deterministic=False, prescaled: bool = False):
        logits, value = self._forward(obs, prescaled)
        logp_all, probs = _categorical(logits)
        action = _sample_or_argmax(logits, logp_all, probs, deterministic)
        logp = logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1)
        return action, logp, value

    def evaluate(self, obs, actions, prescaled: bool = False):
        logits, value = self._forward(obs, prescaled)
        logp_all, probs = _categorical(logits)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        return logp, _entropy(logp_all, probs), value


class MLPActorCritic(nn.Module):
    """Flat-observation variant (actor_critic.py:66-99), used when scenario.yaml sets flatten."""

    def __init__(self, obs_dim, act_dim, hidden_dim=64):
        super().__init__()
        self.actor = nn.Sequential(layer_init(nn.Linear(obs_dim, hidden_dim)), nn.Tanh(),
                                   layer_init(nn.Linear(hidden_dim, hidden_dim)), nn.Tanh(),
                                   layer_init(nn.Linear(hidden_dim, act_dim), std=0.01))
        self.critic = nn.Sequential(layer_init(nn.Linear(obs_dim, hidden_dim)), nn.Tanh(),
                                    layer_init(nn.Linear(hidden_dim, hidden_dim)), nn.Tanh(),
                                    layer_init(nn.Linear(hidden_dim, 1), std=1.0))

    def act(self, obs, deterministic=False, prescaled: bool = False):
        logits = self.actor(obs)
        logp_all, probs = _categorical(logits)
        action = _sample_or_argmax(logits, logp_all, probs, deterministic)
        logp = logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1)
        return action, logp, self.critic(obs).squeeze(-1)

    def evaluate(self, obs, actions, prescaled: bool = False):
        logits = self.actor(obs)
        logp_all, probs = _categorical(logits)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        return logp, _entropy(logp_all, probs), self.critic(obs).squeeze(-1)
