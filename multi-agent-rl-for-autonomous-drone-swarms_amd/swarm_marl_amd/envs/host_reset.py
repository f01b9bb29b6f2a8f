"""Seeded host-side reset draws that reproduce the reference's NumPy random stream.

The in-kernel reset (swarm_reset / auto-reset) uses a counter-based Philox stream instead; these
host draws exist so that `reset(seed=s)` of the dict-API envs yields the exact episodes the
reference yields for the same seed.  Draw order and ranges:
  DroneSwarmEnv.reset     drone_swarm_env.py:72-80 : positions (N,3), goal (3), obstacles (M,3),
                          each U(-W/2, W/2) in float64 then cast to float32.
  SingleDroneEnv.reset    single_drone_env.py:58-66 : position (3), goal (3), obstacles (M,3).
  DronePhysicsEnv.reset   drone_physics_env.py:205-242: per drone pos (3) with z=max(1,z),
                          mass U(0.9,1.1), damping U(0.8,1.2); per obstacle pos (3) with
                          z=max(0.5,z); goal (3) then goal z ~ U(0.5, 2.0).
"""
from __future__ import annotations

import numpy as np


def swarm_reset_draws(rng: np.random.Generator, num_drones: int, num_obstacles: int,
                      world_size: float):
    half = world_size / 2.0
    pos = rng.uniform(-half, half, size=(num_drones, 3)).astype(np.float32)
    goal = rng.uniform(-half, half, size=3).astype(np.float32)
    obst = rng.uniform(-half, half, size=(num_obstacles, 3)).astype(np.float32)
    return pos, goal, obst


def physics_reset_draws(rng: np.random.Generator, num_drones: int, num_obstacles: int,
                        world_size: float):
    half = world_size / 2.0
    pos = np.empty((num_drones, 3), np.float64)
    mass = np.empty(num_drones, np.float64)
    damping = np.empty(num_drones, np.float64)
    for i in range(num_drones):
        p = rng.uniform(-half, half, size=3)
        p[2] = max(1.0, p[2])
        pos[i] = p
        mass[i] = rng.uniform(0.9, 1.1)
        damping[i] = 0.5 * rng.uniform(0.8, 1.2)  # linearDamping = 0.5 * U(0.8, 1.2)
    obst = np.empty((num_obstacles, 3), np.float64)
    for m in range(num_obstacles):
        o = rng.uniform(-half, half, size=3)
        o[2] = max(0.5, o[2])
        obst[m] = o
    goal = rng.uniform(-half, half, size=3).astype(np.float32)
    goal[2] = rng.uniform(0.5, 2.0)
    return (pos.astype(np.float32), goal, obst.astype(np.float32),
            damping.astype(np.float32), mass.astype(np.float32))
