"""SingleDroneEnv — gym.Env drop-in (src/swarm_marl/envs/single_drone_env.py:12-159).

It is the N=1, K=0 case of the swarm kernel: obs = [pos | vel | goal-pos | Ms x obstacle], dim
9 + 4*Ms (:33).  Differences from the swarm env that live in this adapter: the drone keeps
stepping after a termination (no agent removal), and truncated = step_count >= max_steps
independently of terminated (:102-103).
"""
from __future__ import annotations

from dataclasses import replace
from typing import Any

import numpy as np
import torch

from .. import _native as nat
from ..vec_env import VecSwarm
from .common import Box, DroneEnvConfig, GymEnv
from .drone_swarm_env import PackedIO, _host
from .host_reset import swarm_reset_draws


class SingleDroneEnv(GymEnv):
    metadata = {"render_modes": []}

    def __init__(self, config: dict[str, Any] | None = None):
        super().__init__()
        self.cfg = DroneEnvConfig.from_dict(config)
        self.rng = np.random.default_rng(self.cfg.seed)
        self._obs_dim = 9 + 4 * max(self.cfg.sensed_obstacles, 0)
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(self._obs_dim,),
                                     dtype=np.float32)
        self.action_space = Box(low=-1.0, high=1.0, shape=(3,), dtype=np.float32)
        self.step_count = 0
        self._vec = VecSwarm(1, replace(self.cfg, neighbor_k=0, max_steps=2 ** 31 - 1),
                             num_drones=1, dynamics="kinematic", auto_reset=False,
                             with_infos=True, packed_io="mapped")
        self._io = PackedIO(self._vec)

    @property
    def position(self) -> np.ndarray:
        return _host(self._vec.pos[0, 0])

    @property
    def velocity(self) -> np.ndarray:
        return _host(self._vec.vel[0, 0])

    @property
    def goal(self) -> np.ndarray:
        return _host(self._vec.goal[0])

    @property
    def obstacles(self) -> np.ndarray:
        return _host(self._vec.obstacles[0])

    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        super().reset(seed=seed)
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        pos, goal, obst = swarm_reset_draws(self.rng, 1, self.cfg.num_obstacles,
                                            self.cfg.world_size)
        self.step_count = 0
        self._vec.set_state(pos=pos[None], vel=np.zeros((1, 1, 3), np.float32), goal=goal[None],
                            obstacles=obst[None], active=np.ones((1, 1), bool),
                            step_count=np.zeros(1, np.int32))
        self._vec.observe()
        h = self._io.fetch()
        return h["obs"][0, 0].copy(), {"distance_to_goal": float(h["dist_goal"][0, 0])}

    def step(self, action):
        io, v = self._io, self._vec
        io.h_in["actions"][0, 0] = np.asarray(action, np.float32).reshape(3)
        io.h_in["active"][0, 0] = True  # the single drone never leaves the env
        io.send()
        v.step(v.actions_in)
        self.step_count += 1
        h = io.fetch()
        obs = h["obs"][0, 0].copy()
        rew = float(h["reward"][0, 0])
        fl = int(h["info_flags"][0, 0])
        dist = float(h["dist_goal"][0, 0])
        reached = bool(fl & nat.AGENT_REACHED)
        collision = bool(fl & nat.AGENT_COLLISION)
        terminated = bool(reached or collision)
        truncated = bool(self.step_count >= self.cfg.max_steps)
        return obs, rew, terminated, truncated, {"distance_to_goal": dist,
                                                 "reached_goal": reached, "collision": collision}
