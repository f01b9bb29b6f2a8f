"""RLlib batched-env bridge and device global_state consumer.

`SwarmBaseEnv` puts E reference-semantics swarm envs (DroneSwarmEnv, drone_swarm_env.py:92-174)
behind RLlib's `BaseEnv` polling interface, so an RLlib env runner steps all E of them with ONE
kernel launch, one packed H2D copy of the actions and one packed D2H copy of every output,
instead of E MultiAgentEnv objects each paying a launch and a round trip per step:

    env = SwarmBaseEnv(1024, {"num_drones": 4, "seed": 0})
    obs, rew, term, trunc, infos, _ = env.poll()          # MultiEnvDicts {env_id: {agent_id: x}}
    env.send_actions({e: {a: act for a in obs[e]} for e in obs})
    ...
    env.try_reset(e)                                       # after terminateds[e]["__all__"]

Episodes end exactly as in the reference; the next episode is drawn in the same launch (device
Philox, keyed by the global env index and episode), and `try_reset` hands out its first
observation — the reference emits no observation on a terminal step (drone_swarm_env.py:154),
so the in-kernel reset loses nothing.

CTDE global_state (callbacks.py:14-57): the reference copies the (6N+3)-float global state into
every agent's info at every step and the `GlobalStateCallback` stacks those copies.  With
`global_state="device"` the bridge keeps the per-step [E, 6N+3] buffer in a device ring instead
and each info carries a 3-int reference; `DeviceGlobalStateCallback` resolves a trajectory's
references with one device gather and one copy to the host.  `global_state="info"` reproduces
the reference's per-agent copies (for its own GlobalStateCallback).
"""
from __future__ import annotations

import itertools
import weakref
from typing import Any

import numpy as np
import torch

from . import _native as nat
from .envs.common import Box
from .envs.drone_swarm_env import PackedIO, build_step_dicts
from .vec_env import VecSwarm

try:  # RLlib's classes when ray is importable; interface stand-ins otherwise
    from ray.rllib.env.base_env import BaseEnv as _BaseEnv  # type: ignore
except Exception:  # pragma: no cover - ray is absent in this image
    class _BaseEnv:  # type: ignore[no-redef]
        """Interface of ray.rllib.env.base_env.BaseEnv used by the env runners."""

        def poll(self):
            raise NotImplementedError

        def send_actions(self, action_dict):
            raise NotImplementedError

        def try_reset(self, env_id=None, *, seed=None, options=None):
            return None, None

        def get_sub_environments(self, as_dict: bool = False):
            return {} if as_dict else []

        def stop(self) -> None:
            pass

try:
    from ray.rllib.algorithms.callbacks import DefaultCallbacks as _DefaultCallbacks  # type: ignore
except Exception:  # pragma: no cover
    class _DefaultCallbacks:  # type: ignore[no-redef]
        pass

_BRIDGES: "weakref.WeakValueDictionary[int, SwarmBaseEnv]" = weakref.WeakValueDictionary()
_IDS = itertools.count(1)


def pack_actions(action_dict: dict, agent_index: dict, out: np.ndarray) -> None:
    """Nested {env_id: {agent_id: action}} -> out [E, N, 3] float32 (missing -> 0, unknown agent
    ids ignored, like drone_swarm_env.py:103-104)."""
    out.fill(0.0)
    for e, acts in action_dict.items():
        row = out[int(e)]
        for a, v in acts.items():
            i = agent_index.get(a)
            if i is not None:
                row[i] = np.asarray(v, np.float32).reshape(3)


def next_active(info_flags: np.ndarray, env_done: np.ndarray) -> np.ndarray:
    """Agents that continue after a step: those the kernel gave an observation (AGENT_HAS_OBS);
    every agent of an env that was reset in the launch."""
    act = (info_flags & nat.AGENT_HAS_OBS) != 0
    act[(env_done & nat.ENV_RESET) != 0] = True
    return act


class SwarmBaseEnv(_BaseEnv):
    def __init__(self, num_envs: int, config: dict[str, Any] | None = None, *,
                 device: str | torch.device | None = None, seed: int = 0, env_offset: int = 0,
                 global_state: str | None = "info", ring_len: int = 1024):
        raw = dict(config or {})
        if global_state not in ("info", "device", None):
            raise ValueError(f"global_state must be 'info', 'device' or None, got {global_state!r}")
        self.vec = VecSwarm(num_envs, raw, device=device, auto_reset=True, seed=seed,
                            env_offset=env_offset, with_infos=True, with_global_state=True,
                            packed_io=True)
        self.io = PackedIO(self.vec)
        self.num_envs = int(num_envs)
        self.num_drones = self.vec.num_drones
        self.agent_ids = [f"drone_{i}" for i in range(self.num_drones)]
        self.agent_id_to_index = {a: i for i, a in enumerate(self.agent_ids)}
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(self.vec.obs_dim,),
                                     dtype=np.float32)
        self.action_space = Box(low=-1.0, high=1.0, shape=(3,), dtype=np.float32)
        self.global_state_mode = global_state
        self.ring_len = int(ring_len)
        self.gs_dim = 6 * self.num_drones + 3
        self.gs_ring = (torch.empty((self.ring_len, self.num_envs, self.gs_dim), dtype=torch.float32,
                                    device=self.vec.device) if global_state == "device" else None)
        self.id = next(_IDS)
        _BRIDGES[self.id] = self
        self.step_id = 0
        self._pending: dict[int, tuple[dict, dict]] = {}
        self.vec.reset()
        self._active = np.ones((self.num_envs, self.num_drones), bool)
        h = self._fetch()
        self._last = self._initial_poll(h)

    # ------------------------------------------------------------------ plumbing
    def _fetch(self) -> dict[str, np.ndarray]:
        if self.gs_ring is not None:
            self.gs_ring[self.step_id % self.ring_len].copy_(self.vec.global_state)
        return self.io.fetch()

    def _gs_info(self, h, e: int):
        if self.global_state_mode == "info":
            return {"global_state": np.array(h["global_state"][e], dtype=np.float32)}
        if self.global_state_mode == "device":
            return {"global_state_ref": (self.id, self.step_id, e)}
        return {}

    def _reset_dicts(self, h, e: int) -> tuple[dict, dict]:
        obs = {a: np.array(h["obs"][e, i], dtype=np.float32) for i, a in enumerate(self.agent_ids)}
        infos = {a: {"distance_to_goal": float(h["dist_goal"][e, i]), **self._gs_info(h, e)}
                 for i, a in enumerate(self.agent_ids)}
        return obs, infos

    def _initial_poll(self, h):
        obs, infos = {}, {}
        for e in range(self.num_envs):
            obs[e], infos[e] = self._reset_dicts(h, e)
        empty = {e: {} for e in range(self.num_envs)}
        return obs, dict(empty), {e: {"__all__": False} for e in empty}, \
            {e: {"__all__": False} for e in empty}, infos, dict(empty)

    # ------------------------------------------------------------------ BaseEnv API
    def poll(self):
        """(obs, rewards, terminateds, truncateds, infos, off_policy_actions) of the last step
        (the reset observations before the first send_actions)."""
        out, self._last = self._last, ({}, {}, {}, {}, {}, {})
        return out

    def send_actions(self, action_dict: dict) -> None:
        """One step of every env in one launch; envs without actions step with zero actions
        for their active agents, like a reference env stepped with an empty dict."""
        hin = self.io.h_in
        pack_actions(action_dict, self.agent_id_to_index, hin["actions"])
        np.copyto(hin["active"], self._active)
        self.io.send()
        self.vec.step(self.vec.actions_in)
        self.step_id += 1
        h = self._fetch()
        env_done = h["env_done"]
        res = ({}, {}, {}, {}, {}, {})
        for e in range(self.num_envs):
            o, r, te, tr, inf = build_step_dicts(self.agent_ids, h["obs"][e], h["reward"][e],
                                                 h["terminated"][e], h["truncated"][e],
                                                 h["info_flags"][e], h["dist_goal"][e],
                                                 h["global_state"][e], int(env_done[e]),
                                                 gs_info=None if self.global_state_mode == "info"
                                                 else self._gs_info(h, e))
            if env_done[e] & nat.ENV_RESET:
                self._pending[e] = self._reset_dicts(h, e)
            res[0][e], res[1][e], res[2][e], res[3][e], res[4][e] = o, r, te, tr, inf
            res[5][e] = {}
        self._active = next_active(h["info_flags"], env_done)
        self._last = res

    def try_reset(self, env_id=None, *, seed=None, options=None):
        """The next episode's first (obs, infos) for `env_id`: drawn in-kernel at the end of
        its terminal step, or drawn now (device reset of that env) mid-episode."""
        ids = range(self.num_envs) if env_id is None else [int(env_id)]
        obs, infos = {}, {}
        todo = [e for e in ids if e not in self._pending]
        if todo:
            mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.vec.device)
            mask[todo] = 1
            self.vec.reset(mask)
            self.step_id += 1  # a fresh ring slot: refs of the previous step stay valid
            h = self._fetch()
            for e in todo:
                self._pending[e] = self._reset_dicts(h, e)
                self._active[e] = True
        for e in ids:
            obs[e], infos[e] = self._pending.pop(e)
        return obs, infos

    def get_sub_environments(self, as_dict: bool = False):
        return {} if as_dict else []  # the envs live on the device, not as Python objects

    def get_agent_ids(self) -> set:
        return set(self.agent_ids)

    # ------------------------------------------------------------------ global_state ring
    def gather_global_state(self, refs) -> np.ndarray:
        """Rows of the device global_state ring for [(bridge_id, step_id, env_id)] refs."""
        if self.gs_ring is None:
            raise ValueError("bridge was not built with global_state='device'")
        st = np.array([r[1] for r in refs], np.int64)
        ev = np.array([r[2] for r in refs], np.int64)
        if len(st) and (st.min() <= self.step_id - self.ring_len or st.max() > self.step_id):
            raise ValueError(f"global_state refs span steps {st.min()}..{st.max()}, the ring holds "
                             f"{self.step_id - self.ring_len + 1}..{self.step_id} (raise ring_len)")
        slot = torch.as_tensor(st % self.ring_len, device=self.vec.device)
        env = torch.as_tensor(ev, device=self.vec.device)
        return self.gs_ring[slot, env].cpu().numpy()


def resolve_global_state(refs) -> np.ndarray:
    """Stack the global states of a trajectory's references (any mix of bridges)."""
    out = None
    by_bridge: dict[int, list[int]] = {}
    for k, r in enumerate(refs):
        by_bridge.setdefault(int(r[0]), []).append(k)
    for bid, rows in by_bridge.items():
        br = _BRIDGES.get(bid)
        if br is None:
            raise ValueError(f"global_state ref to a bridge that no longer exists ({bid})")
        vals = br.gather_global_state([refs[k] for k in rows])
        if out is None:
            out = np.zeros((len(refs), vals.shape[1]), np.float32)
        out[rows] = vals
    return out if out is not None else np.zeros((0, 0), np.float32)


class DeviceGlobalStateCallback(_DefaultCallbacks):
    """callbacks.py:14-57 GlobalStateCallback, reading the bridge's device ring: fills
    postprocessed_batch["global_state"] ([count, 6N+3] float32) from the infos' references (or
    from per-agent copies, as the reference does, when the infos carry arrays)."""

    def on_postprocess_trajectory(self, *, worker: Any = None, episode: Any = None,
                                  agent_id: str | None = None, policy_id: str | None = None,
                                  policies: dict | None = None, postprocessed_batch: Any = None,
                                  original_batches: dict | None = None, **kwargs) -> None:
        batch = postprocessed_batch
        model = policies[policy_id].model if policies and policy_id in policies else None
        gdim = getattr(model, "global_state_dim", None)
        count = int(getattr(batch, "count", 0) or len(batch.get("infos", [])))
        if gdim:
            batch["global_state"] = np.zeros((count, gdim), dtype=np.float32)
        infos = batch.get("infos") if hasattr(batch, "get") else None
        if infos is None or len(infos) == 0:
            return
        if "global_state" in infos[0]:
            batch["global_state"] = np.array([i["global_state"] for i in infos], dtype=np.float32)
        elif "global_state_ref" in infos[0]:
            batch["global_state"] = resolve_global_state([i["global_state_ref"] for i in infos])
