"""DronePhysicsEnv — dict-API drop-in for the reference PyBullet env, as a GPU point-mass model.

Surface of src/swarm_marl/envs/drone_physics_env.py:22-419 (constructor, reset, set_goal, step,
observation/action spaces, obs layout with the velocity clamped in the obs only).  The dynamics
are the point-mass restatement of the force/substep loop (:320-360): per substep the commanded
acceleration action*max_accel, gravity compensation +9.5 m/s^2, gravity -9.81 m/s^2, linear
damping of the Featherstone base (-d*(1+|v|)*v, or btRigidBody v*=(1-d)^h), semi-implicit Euler,
velocity clamped to max_speed before each substep for agents that supplied an action.  Contacts
are approximated by radii: the rigid-body contact solver, GUI and URDF loading of
PyBullet are not reproduced.  Parity with PyBullet is UNPINNED (pybullet is not installed).
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .. import _native as nat
from ..vec_env import VecSwarm
from .common import Box, DroneEnvConfig, MultiAgentEnv
from .drone_swarm_env import PackedIO, _host
from .host_reset import physics_reset_draws


class DronePhysicsEnv(MultiAgentEnv):
    def __init__(self, config: dict[str, Any] | None = None, *, physics: dict | None = None):
        super().__init__()
        raw = dict(config or {})
        self.num_drones = int(raw.get("num_drones", 3))
        self.cfg = DroneEnvConfig.from_dict({k: v for k, v in raw.items() if k != "num_drones"})
        self.gui = bool(raw.get("gui", False))  # accepted; there is no GUI in this build
        self.action_space = Box(low=-1.0, high=1.0, shape=(3,), dtype=np.float32)
        self._obs_dim = self.cfg.obs_dim()
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(self._obs_dim,),
                                     dtype=np.float32)
        self.agent_ids = [f"drone_{i}" for i in range(self.num_drones)]
        self.agent_id_to_index = {a: i for i, a in enumerate(self.agent_ids)}
        self.agents = list(self.agent_ids)
        self.step_count = 0
        self.rng = np.random.default_rng(self.cfg.seed)
        self.masses = np.ones(self.num_drones, np.float32)
        self._vec = VecSwarm(1, self.cfg, num_drones=self.num_drones, dynamics="physics",
                             auto_reset=False, with_infos=True, with_global_state=True,
                             physics=physics, packed_io="mapped")
        self._io = PackedIO(self._vec)

    @property
    def goal(self) -> np.ndarray:
        return _host(self._vec.goal[0])

    @goal.setter
    def goal(self, v) -> None:
        self._vec.goal[0].copy_(torch.as_tensor(np.asarray(v, np.float32)))

    @property
    def positions(self) -> np.ndarray:
        return _host(self._vec.pos[0])

    @property
    def velocities(self) -> np.ndarray:
        return _host(self._vec.vel[0])

    @property
    def obstacles(self) -> np.ndarray:
        return _host(self._vec.obstacles[0])

    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        # :190-193 — a fresh entropy stream when no seed is given
        self.rng = np.random.default_rng(seed) if seed is not None else np.random.default_rng()
        pos, goal, obst, damping, mass = physics_reset_draws(
            self.rng, self.num_drones, self.cfg.num_obstacles, self.cfg.world_size)
        self.masses = mass  # mass cancels in the point-mass force model
        self.agents = list(self.agent_ids)
        self.step_count = 0
        n = self.num_drones
        self._vec.set_state(pos=pos[None], vel=np.zeros((1, n, 3), np.float32), goal=goal[None],
                            obstacles=obst[None], active=np.ones((1, n), bool),
                            step_count=np.zeros(1, np.int32), damping=damping[None])
        self._vec.observe()
        h = self._io.fetch()
        obs, dist = h["obs"][0], h["dist_goal"][0]
        observations = {a: obs[i].copy() for i, a in enumerate(self.agent_ids)}
        infos = {a: {"distance_to_goal": float(dist[i]), "reached_goal": False, "collision": False}
                 for i, a in enumerate(self.agent_ids)}
        return observations, infos

    def set_goal(self, new_pos) -> None:
        """drone_physics_env.py:265-277 — move the goal (dashboard drag)."""
        self.goal = np.asarray(new_pos, np.float32)

    def step(self, action_dict: dict[str, Any]):
        io, v = self._io, self._vec
        acts, mask, act = io.h_in["actions"][0], io.h_in["action_mask"][0], io.h_in["active"][0]
        acts.fill(0.0)
        mask.fill(0)
        act.fill(False)
        for aid, a in action_dict.items():
            idx = self.agent_ids.index(aid)  # unknown id -> ValueError, as :326
            acts[idx] = np.asarray(a, np.float32).reshape(3)  # no action clip (:336)
            mask[idx] = 1
        for a in self.agents:
            act[self.agent_id_to_index[a]] = True
        io.send()
        v.step(v.actions_in, v.action_mask_in)
        self.step_count += 1
        h = io.fetch()
        obs, rew, dist, flags = h["obs"][0], h["reward"][0], h["dist_goal"][0], h["info_flags"][0]
        gs = h["global_state"][0]
        env_done = int(h["env_done"][0])
        observations = {a: obs[i].copy() for i, a in enumerate(self.agent_ids)}  # all agents
        rewards = {a: float(rew[self.agent_id_to_index[a]]) for a in self.agents}
        term_all = bool(env_done & nat.ENV_TERMINATED)
        trunc_all = bool(env_done & nat.ENV_TRUNCATED)
        terminated = {a: term_all for a in self.agent_ids}
        truncated = {a: trunc_all for a in self.agent_ids}
        terminated["__all__"] = term_all
        truncated["__all__"] = trunc_all
        infos = {}
        for i, a in enumerate(self.agent_ids):
            infos[a] = {"global_state": gs.copy(), "distance_to_goal": float(dist[i]),
                        "reached_goal": bool(dist[i] < self.cfg.goal_radius),
                        "collision": bool(flags[i] & nat.AGENT_COLLISION)}
        if term_all or trunc_all:
            self.agents = []
        return observations, rewards, terminated, truncated, infos
