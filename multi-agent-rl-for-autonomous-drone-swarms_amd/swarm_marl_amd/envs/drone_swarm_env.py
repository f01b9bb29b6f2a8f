"""DroneSwarmEnv — drop-in for the reference RLlib MultiAgentEnv, stepped on the MI355X.

Same constructor, attributes and dict API as src/swarm_marl/envs/drone_swarm_env.py:17-174:
  DroneSwarmEnv(config) ; reset(*, seed=None, options=None) -> (obs, infos)
  step(action_dict) -> (obs, rewards, terminated, truncated, infos)
so `register_env(name, lambda cfg: DroneSwarmEnv(cfg))` in the reference's train_*.py scripts
works unchanged.  Behind the dict surface one env is a VecSwarm of E=1 on the GPU: the whole
step (integrate, distances, collision, formation, rewards, kNN observation) is one kernel launch;
only the dict assembly stays on the host.

Seeded resets draw from numpy.random.default_rng exactly like the reference (host_reset.py), so
the same seeds give the same episodes; rewards are float32-accurate (|err| < 1e-5).
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .. import _native as nat
from ..vec_env import VecSwarm
from .common import Box, DroneEnvConfig, MultiAgentEnv
from .host_reset import swarm_reset_draws


def _host(t: torch.Tensor) -> np.ndarray:
    return t.detach().to("cpu").numpy()


class DroneSwarmEnv(MultiAgentEnv):
    """Multi-agent 3D swarm env; local observations (own pos/vel, goal vector, K nearest
    neighbours, Ms nearest obstacles)."""

    def __init__(self, config: dict[str, Any] | None = None):
        super().__init__()
        raw = dict(config or {})
        self.num_drones = int(raw.get("num_drones", 3))
        self.cfg = DroneEnvConfig.from_dict({k: v for k, v in raw.items() if k != "num_drones"})
        self.rng = np.random.default_rng(self.cfg.seed)
        self.agent_ids = [f"drone_{i}" for i in range(self.num_drones)]
        self.agent_id_to_index = {a: i for i, a in enumerate(self.agent_ids)}
        self.agents = list(self.agent_ids)
        self._obs_dim = self.cfg.obs_dim()
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(self._obs_dim,),
                                     dtype=np.float32)
        self.action_space = Box(low=-1.0, high=1.0, shape=(3,), dtype=np.float32)
        self._vec = VecSwarm(1, self.cfg, num_drones=self.num_drones, dynamics="kinematic",
                             auto_reset=False, with_infos=True, with_global_state=True)
        self._vec.active.fill_(True)

    # ---- state attributes read (and written) by callers: visualize_swarm.py:76-110 ----------
    @property
    def positions(self) -> np.ndarray:
        return _host(self._vec.pos[0])

    @positions.setter
    def positions(self, v) -> None:
        self._vec.pos[0].copy_(torch.as_tensor(np.asarray(v, np.float32)))

    @property
    def velocities(self) -> np.ndarray:
        return _host(self._vec.vel[0])

    @velocities.setter
    def velocities(self, v) -> None:
        self._vec.vel[0].copy_(torch.as_tensor(np.asarray(v, np.float32)))

    @property
    def goal(self) -> np.ndarray:
        return _host(self._vec.goal[0])

    @goal.setter
    def goal(self, v) -> None:
        self._vec.goal[0].copy_(torch.as_tensor(np.asarray(v, np.float32)))

    @property
    def obstacles(self) -> np.ndarray:
        return _host(self._vec.obstacles[0])

    @obstacles.setter
    def obstacles(self, v) -> None:
        self._vec.obstacles[0].copy_(torch.as_tensor(np.asarray(v, np.float32)))

    @property
    def step_count(self) -> int:
        return int(self._vec.step_count[0].item())

    @step_count.setter
    def step_count(self, v: int) -> None:
        self._vec.step_count[0] = int(v)

    def _sync_active(self) -> None:
        mask = np.zeros(self.num_drones, bool)
        for a in self.agents:
            mask[self.agent_id_to_index[a]] = True
        self._vec.active[0].copy_(torch.as_tensor(mask))

    # ---- API -------------------------------------------------------------------------------
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        pos, goal, obst = swarm_reset_draws(self.rng, self.num_drones, self.cfg.num_obstacles,
                                            self.cfg.world_size)
        self.agents = list(self.agent_ids)
        v = self._vec
        v.set_state(pos=pos[None], vel=np.zeros((1, self.num_drones, 3), np.float32),
                    goal=goal[None], obstacles=obst[None], active=np.ones((1, self.num_drones), bool),
                    step_count=np.zeros(1, np.int32))
        v.observe()
        obs = _host(v.obs[0])
        dist = _host(v.dist_goal[0])
        gs = _host(v.global_state[0])
        observations = {a: obs[i].copy() for i, a in enumerate(self.agent_ids)}
        infos = {a: {"distance_to_goal": float(dist[i]), "global_state": gs.copy()}
                 for i, a in enumerate(self.agent_ids)}
        return observations, infos

    def step(self, action_dict: dict[str, Any]):
        if not self.agents:  # drone_swarm_env.py:93-95
            return {}, {}, {"__all__": True}, {"__all__": False}, {}
        self._sync_active()
        acts = np.zeros((1, self.num_drones, 3), np.float32)
        for a in self.agents:  # missing -> zero action, unknown ids ignored (:103-104)
            if a in action_dict:
                acts[0, self.agent_id_to_index[a]] = np.asarray(action_dict[a], np.float32).reshape(3)
        v = self._vec
        v.step(torch.as_tensor(acts).to(v.device))
        return self._collect()

    def _collect(self):
        v = self._vec
        packed = torch.cat([v.obs[0].reshape(-1), v.reward[0], v.dist_goal[0],
                            v.global_state[0]]).to("cpu").numpy()
        flags = _host(torch.stack([v.terminated[0].to(torch.uint8), v.truncated[0].to(torch.uint8),
                                   v.info_flags[0]]))
        env_done = int(v.env_done[0].item())
        n, d = self.num_drones, self._obs_dim
        obs = packed[: n * d].reshape(n, d)
        rew = packed[n * d: n * d + n]
        dist = packed[n * d + n: n * d + 2 * n]
        gs = packed[n * d + 2 * n:]
        return build_step_dicts(self.agent_ids, obs, rew, flags[0], flags[1], flags[2], dist, gs,
                                env_done, self)


def build_step_dicts(agent_ids, obs, rew, term, trunc, info_flags, dist, gs, env_done, env=None):
    """Assemble the RLlib dicts from the kernel's dense outputs (drone_swarm_env.py:129-174).

    Pure host logic on numpy arrays; `env.agents` is updated when an env is given.
    """
    rewards, terminated, truncated, infos, observations = {}, {}, {}, {}, {}
    nxt = []
    for i, a in enumerate(agent_ids):
        fl = int(info_flags[i])
        if not fl & nat.AGENT_STEPPED:
            continue
        rewards[a] = float(rew[i])
        terminated[a] = bool(term[i])
        truncated[a] = bool(trunc[i])
        if fl & nat.AGENT_HAS_OBS:
            observations[a] = np.array(obs[i], dtype=np.float32)
            infos[a] = {"distance_to_goal": float(dist[i]),
                        "reached_goal": bool(fl & nat.AGENT_REACHED),
                        "collision": bool(fl & nat.AGENT_COLLISION),
                        "global_state": np.array(gs, dtype=np.float32)}
            nxt.append(a)
    terminated["__all__"] = bool(env_done & nat.ENV_TERMINATED)
    truncated["__all__"] = bool(env_done & nat.ENV_TRUNCATED)
    if env is not None:
        env.agents = [] if (terminated["__all__"] or truncated["__all__"]) else nxt
    return observations, rewards, terminated, truncated, infos
