"""Environment package: the reference's env classes backed by the MI355X swarm kernel.

Mirrors `swarm_marl.envs` (src/swarm_marl/envs/__init__.py:3-6) plus DronePhysicsEnv.
"""
from .common import DroneEnvConfig
from .drone_physics_env import DronePhysicsEnv
from .drone_swarm_env import DroneSwarmEnv
from .single_drone_env import SingleDroneEnv

__all__ = ["DroneEnvConfig", "DroneSwarmEnv", "DronePhysicsEnv", "SingleDroneEnv"]
