"""CPU oracle for per-env parameters (swarm_env_cfg_t) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module; the
product path never does.

A batch whose envs carry their own parameters must behave, env by env, exactly like a batch of
one env whose uniform config holds those values (the reference has one config per env instance:
DroneSwarmEnv(config) at drone_swarm_env.py:28-63; curriculum stages build a new env_config per
stage, scripts/train_curriculum.py:159-233).  So the oracle steps every env on its own through
swarm_oracle.step with that env's config (global env index as env_offset, so the device reset
draws are the same), and a reset draws the new episode with the NEXT episode's config when one is
given (the device copies env_cfg_next into env_cfg before drawing).  Obstacle slots beyond an
env's count are zero, as the device stores them.
"""
from __future__ import annotations

import numpy as np

from . import swarm_oracle as so

f32 = np.float32

OVERRIDES = ("world_size", "dt", "max_speed", "max_accel", "obstacle_radius", "max_steps", "num_obstacles")


def env_cfg(base: dict, over: dict | None, e: int) -> dict:
    """base config with env e's overrides (scalars or per-env sequences)."""
    cfg = dict(base)
    for k, v in (over or {}).items():
        if v is None:
            continue
        val = np.asarray(v)
        val = val if val.ndim == 0 else val[e]
        cfg[k] = int(val) if k in ("max_steps", "num_obstacles") else float(val)
    m = int(base["num_obstacles"])
    cfg["num_obstacles"] = min(max(int(cfg["num_obstacles"]), 0), m)
    return cfg


def _slice(state: dict, e: int, m_e: int) -> dict:
    st = {k: np.array(v[e:e + 1], copy=True) for k, v in state.items()}
    st["obst"] = st["obst"][:, :m_e].copy()
    return st


def _merge(dst: dict, src: dict, e: int, m: int) -> None:
    for k, v in src.items():
        if k == "obst":
            row = np.zeros((m, 3), f32)
            row[:v.shape[1]] = v[0]
            dst[k][e] = row
        else:
            dst[k][e] = v[0]


def step(base: dict, cur: dict | None, state: dict, actions, *, nxt: dict | None = None,
         auto_reset: bool = True, seed: int = 0, env_offset: int = 0, physics: bool = False):
    """One step of every env with per-env parameters.  Returns (new_state, out, new_cur) where
    new_cur is the per-env override dict in force after the step (the next-episode values for
    envs that reset).  out holds the swarm_oracle.step fields, stacked over envs."""
    e_n = state["pos"].shape[0]
    m = int(base["num_obstacles"])
    new_state = {k: np.array(v, copy=True) for k, v in state.items()}
    outs = []
    new_cur = {k: (np.array(np.broadcast_to(np.asarray(v), (e_n,)), copy=True) if v is not None else None)
               for k, v in (cur or {}).items()}
    for k, v in (nxt or {}).items():
        if k not in new_cur or new_cur[k] is None:
            new_cur[k] = np.array([env_cfg(base, cur, e)[k] for e in range(e_n)])
    for e in range(e_n):
        cfg_e = env_cfg(base, cur, e)
        st_e = _slice(state, e, cfg_e["num_obstacles"])
        ns, out = so.step(cfg_e, st_e, np.asarray(actions)[e:e + 1], auto_reset=False, seed=seed,
                          env_offset=env_offset + e, physics=physics)
        done = bool(out["term_all"][0] or out["trunc_all"][0])
        out = dict(out)
        out["reset"] = np.array([done and auto_reset])
        if done and auto_reset:
            cfg_n = env_cfg(base, nxt, e) if nxt else cfg_e
            if nxt:
                for k in nxt:
                    new_cur[k][e] = cfg_n[k]
            if cfg_n["num_obstacles"] != ns["obst"].shape[1]:
                ns["obst"] = np.zeros((1, cfg_n["num_obstacles"], 3), f32)
            ns, ro = so.reset_device(cfg_n, ns, seed=seed, env_offset=env_offset + e, physics=physics)
            out["obs"], out["global_state"] = ro["obs"], ro["global_state"]
        _merge(new_state, ns, e, m)
        outs.append(out)
    stacked = {k: np.concatenate([o[k] for o in outs], axis=0) for k in outs[0]}
    return new_state, stacked, new_cur


def reset(base: dict, cur: dict | None, state: dict, *, nxt: dict | None = None, env_mask=None,
          seed: int = 0, env_offset: int = 0, physics: bool = False):
    """swarm_reset of the masked envs (all if None) with per-env parameters (next-episode values
    when given); out rows of envs outside the mask are zero."""
    e_n = state["pos"].shape[0]
    m = int(base["num_obstacles"])
    mask = np.ones(e_n, bool) if env_mask is None else np.asarray(env_mask, bool)
    new_state = {k: np.array(v, copy=True) for k, v in state.items()}
    outs = []
    for e in range(e_n):
        if not mask[e]:
            _, ro = so.reset_device(base, _slice(state, e, 0) | {"obst": np.zeros((1, m, 3), f32)}, seed=seed,
                                    env_offset=env_offset + e, physics=physics)
            outs.append({k: np.zeros_like(v) for k, v in ro.items()})
            continue
        cfg_e = env_cfg(base, nxt if nxt else cur, e)
        st_e = _slice(state, e, cfg_e["num_obstacles"])
        st_e["obst"] = np.zeros((1, cfg_e["num_obstacles"], 3), f32)
        ns, ro = so.reset_device(cfg_e, st_e, seed=seed, env_offset=env_offset + e, physics=physics)
        _merge(new_state, ns, e, m)
        outs.append(ro)
    return new_state, {k: np.concatenate([o[k] for o in outs], axis=0) for k in outs[0]}
