"""YAML -> env factory (src/scenario_creator/scenario_creator.py of the reference).

``ScenarioCreator(config_path).create_env(difficulty, seed)`` returns a single-env
gym-style ``MerlinEnv`` (uint8[56, 56, 3] RGB partial observations, 3 actions) --
the same observation/action contract as the reference's wrapper chain
RGBImgPartialObsWrapper -> ImgObsWrapper -> ThreeActionWrapper (scenario_creator.py:43-55).
Like the reference, ``seed`` does not seed the env (scenario_creator.py:35-57 ignores
it); seed through ``env.reset(seed=...)``.
``create_vec_env(difficulty, num_envs, seed, ...)`` builds the GPU vector env used by
the fast path.  The single env also takes the config's other observation modes
(``fully_observable``: the encoded grid; ``flatten``: the flattened RGB view, PPO's MLP path,
src/ppo.py:38-41); the batched vector env refuses them (its CNN path needs the (56, 56, 3) view).
"""
from __future__ import annotations

import os

import yaml

from .envs import MerlinEnv, MerlinVecEnv

DEFAULT_CONFIG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config", "scenario.yaml")

_ENV_IDS = {
    "MERLIN-Easy-v0": "easy",
    "MERLIN-Medium-v0": "medium",
    "MERLIN-MediumHard-v0": "mediumhard",
    "MERLIN-Hard-v0": "hard",
    "MERLIN-Hardest-v0": "hardest",
}


class ScenarioCreator:
    def __init__(self, config_path: str = DEFAULT_CONFIG):
        if not os.path.exists(config_path):
            raise FileNotFoundError(f"Config not found: {config_path}")
        with open(config_path, "r") as f:
            self.config = yaml.safe_load(f)
        self.seed = self.config.get("seed", 42)
        self.global_cfg = self.config.get("global", {})
        self.obs_cfg = self.config.get("observation", {})
        self.rewards_cfg = self.config.get("rewards", {})
        self.logging_cfg = self.config.get("logging", {})
        self._validate_grid_sizes()

    def _validate_grid_sizes(self):
        sizes = {cfg["env_id"].split("-")[-2] for cfg in self.config["difficulties"].values()
                 if "-" in cfg["env_id"] and "x" in cfg["env_id"]}
        if len(sizes) > 1:
            raise ValueError(f"Multiple grid sizes detected: {sizes}")

    def _env_kwargs(self, difficulty: str) -> dict:
        cfg = self.config["difficulties"].get(difficulty)
        if not cfg:
            raise ValueError(f"Unknown difficulty: {difficulty}")
        kw = {**self.global_cfg, **cfg.get("params", {})}
        kw.pop("render_mode", None)
        gen = _ENV_IDS.get(cfg["env_id"], difficulty)
        return {"difficulty": gen, "size": int(kw.pop("size", 16)), **kw}

    def create_env(self, difficulty: str = "easy", seed=None, device="cuda", **flags):
        """The single env of scenario_creator.py:35-57 with the configured observation wrappers (observation.
        fully_observable: the encoded full grid instead of the RGB partial view; observation.flatten: as a vector)."""
        obs = {"fully_observable": bool(self.obs_cfg.get("fully_observable", False)),
               "flatten": bool(self.obs_cfg.get("flatten", False))}
        return MerlinEnv(device=device, **self._env_kwargs(difficulty), **obs, **flags)

    def create_vec_env(self, difficulty: str, num_envs: int, seed=None, device="cuda", env_offset: int = 0,
                       **flags) -> MerlinVecEnv:
        """N envs for the batched trainer.  Their step produces the RGB partial view's tile codes; with
        observation.flatten the batched trainer takes the reference's MLP path on the flattened view (the RGB view, or
        with observation.fully_observable the encoded full grid: MerlinVecEnv.flat_obs / render_full).  The full grid
        unflattened is refused: it is 16 x 16, smaller than CNNActorCritic's receptive field (the reference's CNN
        fails on it too)."""
        full, flat = bool(self.obs_cfg.get("fully_observable", False)), bool(self.obs_cfg.get("flatten", False))
        if full and not flat:
            raise ValueError("CNNActorCritic trains on the (56, 56, 3) RGB partial view (src/actor_critic.py:22-28); "
                             "observation.fully_observable without flatten gives a grid smaller than its receptive field")
        return MerlinVecEnv(num_envs, seed=seed, device=device, env_offset=env_offset, fully_observable=full,
                            flatten=flat, **self._env_kwargs(difficulty), **flags)

    def sample_scenarios(self, n: int = 5, difficulty: str = "easy"):
        return [self.create_env(difficulty) for _ in range(n)]

    def get_env_id(self, difficulty: str) -> str:
        return self.config["difficulties"][difficulty]["env_id"]

    def get_logging_params(self) -> dict:
        return self.logging_cfg

    def get_observation_params(self) -> dict:
        return self.obs_cfg

    def get_env_size_str(self, difficulty: str) -> str:
        size = self.config["difficulties"][difficulty].get("params", {}).get("size", 16)
        return f"{size}x{size}"
