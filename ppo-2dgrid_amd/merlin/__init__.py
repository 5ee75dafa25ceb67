"""MERLIN-AMD: MI355X-native hot path of PPO-2DGrid (batched MiniGrid + PPO).

Public surface mirrors the reference's ``src`` package (src/__init__.py):
``CNNActorCritic``, ``MLPActorCritic``, ``RolloutBuffer``, ``PPO``, ``ScenarioCreator``,
``get_device``, ``layer_init`` -- plus the GPU envs ``MerlinVecEnv`` / ``MerlinEnv``.
The env dynamics, observation rendering, GAE and advantage normalisation run in
lib/libmerlin_hip.so (HIP, gfx950); there is no CPU fallback.
"""
from .actor_critic import CNNActorCritic, MLPActorCritic
from .envs import MerlinEnv, MerlinVecEnv
from .ppo import PPO
from .rollout_buffer import CodeRolloutBuffer, RolloutBuffer
from .scenario_creator import ScenarioCreator
from .utils.utils import get_device, set_seed
from .utils.utils_rl import compute_gae_standard, layer_init

__all__ = ["CNNActorCritic", "MLPActorCritic", "MerlinEnv", "MerlinVecEnv", "PPO", "CodeRolloutBuffer",
           "RolloutBuffer", "ScenarioCreator", "get_device", "set_seed", "compute_gae_standard", "layer_init"]
