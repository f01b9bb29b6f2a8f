"""DroneSwarmEnv — drop-in for the reference RLlib MultiAgentEnv, stepped on the MI355X.

Same constructor, attributes and dict API as src/swarm_marl/envs/drone_swarm_env.py:17-174:
  DroneSwarmEnv(config) ; reset(*, seed=None, options=None) -> (obs, infos)
  step(action_dict) -> (obs, rewards, terminated, truncated, infos)
so `register_env(name, lambda cfg: DroneSwarmEnv(cfg))` in the reference's train_*.py scripts
works unchanged.  Behind the dict surface one env is a VecSwarm of E=1 on the GPU: the whole
step (integrate, distances, collision, formation, rewards, kNN observation) is one kernel launch;
only the dict assembly stays on the host.  Per step the host fills one pinned input block
(actions + active mask), which goes over in ONE async H2D copy; the kernel writes every output
into one device arena, which comes back in ONE async D2H copy; one stream synchronisation.

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
                             auto_reset=False, with_infos=True, with_global_state=True,
                             packed_io="mapped")
        self._vec.active.fill_(True)
        self._io = PackedIO(self._vec)

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
        h = self._io.fetch()
        obs, dist, gs = h["obs"][0], h["dist_goal"][0], h["global_state"][0]
        observations = {a: obs[i].copy() for i, a in enumerate(self.agent_ids)}
        infos = {a: {"distance_to_goal": float(dist[i]), "global_state": gs.copy()}
                 for i, a in enumerate(self.agent_ids)}
        return observations, infos

    def step(self, action_dict: dict[str, Any]):
        if not self.agents:  # drone_swarm_env.py:93-95
            return {}, {}, {"__all__": True}, {"__all__": False}, {}
        io = self._io
        acts, active = io.h_in["actions"][0], io.h_in["active"][0]
        acts.fill(0.0)
        active.fill(False)
        idx = self.agent_id_to_index
        for a in self.agents:  # missing -> zero action, unknown ids ignored (:103-104)
            i = idx[a]
            active[i] = True
            if a in action_dict:
                acts[i] = np.asarray(action_dict[a], np.float32).reshape(3)
        io.send()
        self._vec.step(self._vec.actions_in)
        h = io.fetch()
        return build_step_dicts(self.agent_ids, h["obs"][0], h["reward"][0], h["terminated"][0],
                                h["truncated"][0], h["info_flags"][0], h["dist_goal"][0],
                                h["global_state"][0], int(h["env_done"][0]), self)


class PackedIO:
    """Pinned host mirrors of a packed_io VecSwarm's input and output arenas: send() is one async
    H2D copy of the inputs, fetch() one async D2H copy of every output plus one stream sync, and
    returns numpy views of the host mirror (overwritten by the next fetch)."""

    def __init__(self, vec: VecSwarm):
        self.vec = vec
        self.mapped = vec.mapped_io
        if self.mapped:  # the arenas are pinned host memory the kernel uses in place: no mirrors
            self._hin, self._hout = vec.in_arena, vec.out_arena
        else:
            self._hin = torch.empty(vec.in_arena.shape, dtype=torch.uint8, pin_memory=True)
            self._hout = torch.empty(vec.out_arena.shape, dtype=torch.uint8, pin_memory=True)
        self.h_in = {k: t.numpy() for k, t in VecSwarm.arena_views(self._hin, vec.in_layout).items()}
        self.h_out = {k: t.numpy() for k, t in VecSwarm.arena_views(self._hout, vec.out_layout).items()}

    def send(self) -> None:
        if not self.mapped:
            self.vec.in_arena.copy_(self._hin, non_blocking=True)

    def fetch(self) -> dict[str, np.ndarray]:
        if not self.mapped:
            self._hout.copy_(self.vec.out_arena, non_blocking=True)
        torch.cuda.current_stream(self.vec.device).synchronize()
        return self.h_out


def build_step_dicts(agent_ids, obs, rew, term, trunc, info_flags, dist, gs, env_done, env=None,
                     gs_info=None):
    """Assemble the RLlib dicts from the kernel's dense outputs (drone_swarm_env.py:129-174).

    Pure host logic on numpy arrays; `env.agents` is updated when an env is given.  Each info
    gets its own copy of `gs` as "global_state" (like the reference), or the entries of
    `gs_info` instead when given (e.g. a device-ring reference; {} for none).
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
                        "collision": bool(fl & nat.AGENT_COLLISION)}
            if gs_info is None:
                infos[a]["global_state"] = np.array(gs, dtype=np.float32)
            else:
                infos[a].update(gs_info)
            nxt.append(a)
    terminated["__all__"] = bool(env_done & nat.ENV_TERMINATED)
    truncated["__all__"] = bool(env_done & nat.ENV_TRUNCATED)
    if env is not None:
        env.agents = [] if (terminated["__all__"] or truncated["__all__"]) else nxt
    return observations, rewards, terminated, truncated, infos
