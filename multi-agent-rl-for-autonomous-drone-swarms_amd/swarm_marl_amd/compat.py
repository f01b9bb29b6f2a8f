"""Opt-in rebinding of the reference package's env classes to this engine.

    import swarm_marl_amd.compat as compat; compat.install()

After install(), `from swarm_marl.envs import DroneSwarmEnv` (and the physics/single-drone
classes) resolve to the MI355X-backed classes, so the reference's scripts/train_*.py
(register_env(name, lambda cfg: DroneSwarmEnv(cfg)), e.g. train_ctde.py:125) run unchanged.
"""
from __future__ import annotations

import importlib
import sys


def install() -> list[str]:
    from .envs import DronePhysicsEnv, DroneSwarmEnv, SingleDroneEnv

    patched = []
    targets = {
        "swarm_marl.envs": {"DroneSwarmEnv": DroneSwarmEnv, "SingleDroneEnv": SingleDroneEnv},
        "swarm_marl.envs.drone_swarm_env": {"DroneSwarmEnv": DroneSwarmEnv},
        "swarm_marl.envs.single_drone_env": {"SingleDroneEnv": SingleDroneEnv},
        "swarm_marl.envs.drone_physics_env": {"DronePhysicsEnv": DronePhysicsEnv},
    }
    for modname, attrs in targets.items():
        try:
            mod = sys.modules.get(modname) or importlib.import_module(modname)
        except Exception:  # reference package (or pybullet for the physics module) absent
            continue
        for k, v in attrs.items():
            setattr(mod, k, v)
            patched.append(f"{modname}.{k}")
    return patched
