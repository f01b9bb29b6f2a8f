"""Environment configuration and the Gymnasium / RLlib base-class shims.

`DroneEnvConfig` keeps the reference's field names, defaults and `from_dict` behaviour
(src/swarm_marl/envs/common.py:7-32): unknown keys are ignored, a falsy dict gives defaults.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Any

import numpy as np


@dataclass
class DroneEnvConfig:
    world_size: float = 20.0
    dt: float = 0.1
    max_steps: int = 400
    max_speed: float = 4.0
    max_accel: float = 2.0
    collision_radius: float = 0.5
    goal_radius: float = 0.8
    num_obstacles: int = 8
    sensed_obstacles: int = 4
    neighbor_k: int = 3
    obstacle_radius: float = 0.8
    desired_spacing: float = 2.5
    reward_progress_scale: float = 2.0
    reward_goal: float = 25.0
    reward_collision: float = -25.0
    reward_formation_scale: float = 0.15
    seed: int | None = None

    @classmethod
    def from_dict(cls, raw: dict[str, Any] | None) -> "DroneEnvConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in (raw or {}).items() if k in names})

    def obs_dim(self, with_neighbors: bool = True) -> int:
        k = max(self.neighbor_k, 0) if with_neighbors else 0
        return 9 + 4 * k + 4 * max(self.sensed_obstacles, 0)


# --- gymnasium.spaces.Box when gymnasium is importable, a minimal stand-in otherwise ---------
try:  # pragma: no cover - depends on the environment
    from gymnasium import spaces as _gym_spaces

    Box = _gym_spaces.Box
    HAVE_GYMNASIUM = True
except ModuleNotFoundError:
    HAVE_GYMNASIUM = False

    class Box:  # type: ignore[no-redef]
        """Subset of gymnasium.spaces.Box used by the envs' callers (shape/dtype/sample)."""

        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.dtype = np.dtype(dtype)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)
            self._rng = np.random.default_rng(seed)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        def __repr__(self) -> str:
            return f"Box({self.shape}, {self.dtype})"


# --- RLlib MultiAgentEnv when ray is importable, a stub otherwise (as drone_swarm_env.py:8-12) --
try:  # pragma: no cover - depends on the environment
    from ray.rllib.env.multi_agent_env import MultiAgentEnv
except ModuleNotFoundError:
    class MultiAgentEnv:  # type: ignore[no-redef]
        pass

try:  # pragma: no cover
    import gymnasium as _gym

    GymEnv = _gym.Env
except ModuleNotFoundError:
    class GymEnv:  # type: ignore[no-redef]
        metadata: dict = {}

        def reset(self, *, seed=None, options=None):
            return None
