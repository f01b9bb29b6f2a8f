"""ctypes front-end of the C oracle (oracle/swarm_oracle.c) — TEST INFRASTRUCTURE ONLY.

Same state/array conventions as oracle/swarm_oracle.py.  Used by tests (cross-check) and by
bench.py's cpu_baseline leg (multi-threaded timing on the host cores).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# SWARM_ORACLE_LIB: another build of the same source (the ASan/UBSan one, tests/test_sanitizers_cpu.py)
LIB_PATH = Path(os.environ.get("SWARM_ORACLE_LIB", HERE / "build" / "libswarm_oracle.so"))


class Params(ctypes.Structure):  # mirror of swarm_params_t (include/swarm_mi355x.h)
    _fields_ = [(n, ctypes.c_int32) for n in (
        "abi_version", "num_envs", "num_drones", "num_obstacles", "sensed_obstacles", "neighbor_k",
        "max_steps", "dynamics", "reward_mode", "auto_reset", "physics_substeps", "damping_law")] + [
        ("env_offset", ctypes.c_int64), ("seed", ctypes.c_uint64)] + [(n, ctypes.c_double) for n in (
            "world_size", "dt", "max_speed", "max_accel", "collision_radius", "goal_radius",
            "obstacle_radius", "desired_spacing", "reward_progress_scale", "reward_goal",
            "reward_collision", "reward_formation_scale", "gravity", "gravity_comp", "substep_dt",
            "drone_contact_radius", "ground_contact_height")] + [
        ("kernel_path", ctypes.c_int32), ("waves_per_simd", ctypes.c_int32)]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(f"{LIB_PATH} missing; run `make -C oracle`")
        _LIB = ctypes.CDLL(str(LIB_PATH))
        _LIB.oracle_run.restype = ctypes.c_int
        _LIB.oracle_max_threads.restype = ctypes.c_int
        _LIB.oracle_philox4x32_10.restype = None
    return _LIB


def make_params(cfg: dict, num_envs: int, *, physics=False, auto_reset=False, seed=0,
                env_offset=0) -> Params:
    p = Params()
    p.abi_version = 3
    p.num_envs = num_envs
    p.num_drones = int(cfg["num_drones"])
    p.num_obstacles = int(cfg["num_obstacles"])
    p.sensed_obstacles = int(cfg["sensed_obstacles"])
    p.neighbor_k = int(cfg["neighbor_k"])
    p.max_steps = int(cfg["max_steps"])
    p.dynamics = 1 if physics else 0
    p.reward_mode = 1 if physics else 0
    p.auto_reset = 1 if auto_reset else 0
    p.physics_substeps = int(cfg.get("physics_substeps", int(float(cfg["dt"]) * 240)))
    p.damping_law = int(cfg.get("damping_law", 0))
    p.env_offset = int(env_offset)
    p.seed = int(seed)
    for n in ("world_size", "dt", "max_speed", "max_accel", "collision_radius", "goal_radius",
              "obstacle_radius", "desired_spacing", "reward_progress_scale", "reward_goal",
              "reward_collision", "reward_formation_scale", "gravity", "gravity_comp",
              "substep_dt", "drone_contact_radius", "ground_contact_height"):
        setattr(p, n, float(cfg[n]))
    return p


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def run(cfg: dict, state: dict, mode: str = "step", actions=None, action_mask=None, env_mask=None,
        *, physics=False, auto_reset=False, seed=0, env_offset=0, nthreads=0):
    """Run one oracle call in place on copies of `state`; returns (new_state, out)."""
    st = dict(
        pos=np.ascontiguousarray(state["pos"], np.float32).copy(),
        vel=np.ascontiguousarray(state["vel"], np.float32).copy(),
        goal=np.ascontiguousarray(state["goal"], np.float32).copy(),
        obst=np.ascontiguousarray(state["obst"], np.float32).copy(),
        active=np.ascontiguousarray(state["active"]).astype(np.uint8),
        step=np.ascontiguousarray(state["step"], np.int32).copy(),
        episode=np.ascontiguousarray(state.get("episode", np.zeros(len(state["pos"]))),
                                     dtype=np.uint32).copy(),
        damping=np.ascontiguousarray(state.get("damping", np.zeros(state["pos"].shape[:2])),
                                     dtype=np.float32).copy(),
    )
    e, n = st["pos"].shape[:2]
    d = 9 + 4 * max(int(cfg["neighbor_k"]), 0) + 4 * max(int(cfg["sensed_obstacles"]), 0)
    out = dict(obs=np.zeros((e, n, d), np.float32), reward=np.zeros((e, n), np.float64),
               terminated=np.zeros((e, n), np.uint8), truncated=np.zeros((e, n), np.uint8),
               env_done=np.zeros(e, np.uint8), dist_goal=np.zeros((e, n), np.float32),
               flags=np.zeros((e, n), np.uint8), global_state=np.zeros((e, 6 * n + 3), np.float32))
    mode_i = {"step": 0, "reset": 1, "observe": 2}[mode]
    acts = None if actions is None else np.ascontiguousarray(actions, np.float32)
    am = None if action_mask is None else np.ascontiguousarray(action_mask).astype(np.uint8)
    em = None if env_mask is None else np.ascontiguousarray(env_mask).astype(np.uint8)
    prm = make_params(cfg, e, physics=physics, auto_reset=auto_reset, seed=seed,
                      env_offset=env_offset)
    rc = lib().oracle_run(
        ctypes.byref(prm), mode_i, _p(st["pos"]), _p(st["vel"]), _p(st["goal"]),
        _p(st["obst"]) if st["obst"].size else None, _p(st["active"]), _p(st["step"]),
        _p(st["episode"]), _p(st["damping"]), _p(acts), _p(am), _p(em), _p(out["obs"]),
        _p(out["reward"]), _p(out["terminated"]), _p(out["truncated"]), _p(out["env_done"]),
        _p(out["dist_goal"]), _p(out["flags"]), _p(out["global_state"]), int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle_run failed")
    st["active"] = st["active"].astype(bool)
    return st, out


def philox4x32_10(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def max_threads() -> int:
    return int(lib().oracle_max_threads())


class Runner:
    """Persistent-buffer stepping of the C oracle (no per-call copies or allocations): the
    bench's CPU-baseline loop.  State arrays are updated in place by every call."""

    def __init__(self, cfg: dict, num_envs: int, *, seed=0, env_offset=0, nthreads=0, physics=False):
        self.cfg, self.e, self.seed, self.nthreads = cfg, int(num_envs), int(seed), int(nthreads)
        n, m = int(cfg["num_drones"]), int(cfg["num_obstacles"])
        d = 9 + 4 * max(int(cfg["neighbor_k"]), 0) + 4 * max(int(cfg["sensed_obstacles"]), 0)
        e = self.e
        self.st = dict(pos=np.zeros((e, n, 3), np.float32), vel=np.zeros((e, n, 3), np.float32),
                       goal=np.zeros((e, 3), np.float32), obst=np.zeros((e, m, 3), np.float32),
                       active=np.ones((e, n), np.uint8), step=np.zeros(e, np.int32),
                       episode=np.zeros(e, np.uint32), damping=np.zeros((e, n), np.float32))
        self.out = dict(obs=np.zeros((e, n, d), np.float32), reward=np.zeros((e, n), np.float64),
                        terminated=np.zeros((e, n), np.uint8), truncated=np.zeros((e, n), np.uint8),
                        env_done=np.zeros(e, np.uint8), dist_goal=np.zeros((e, n), np.float32),
                        flags=np.zeros((e, n), np.uint8),
                        global_state=np.zeros((e, 6 * n + 3), np.float32))
        self.prm = make_params(cfg, e, physics=physics, auto_reset=True, seed=seed, env_offset=env_offset)
        self._call(1, None)  # device-RNG reset of every env

    def _call(self, mode: int, actions) -> None:
        st, out = self.st, self.out
        rc = lib().oracle_run(
            ctypes.byref(self.prm), mode, _p(st["pos"]), _p(st["vel"]), _p(st["goal"]),
            _p(st["obst"]) if st["obst"].size else None, _p(st["active"]), _p(st["step"]),
            _p(st["episode"]), _p(st["damping"]), _p(actions), None, None, _p(out["obs"]),
            _p(out["reward"]), _p(out["terminated"]), _p(out["truncated"]), _p(out["env_done"]),
            _p(out["dist_goal"]), _p(out["flags"]), _p(out["global_state"]), self.nthreads)
        if rc != 0:
            raise RuntimeError("oracle_run failed")

    def step(self, actions: np.ndarray) -> None:
        self._call(0, np.ascontiguousarray(actions, np.float32))
