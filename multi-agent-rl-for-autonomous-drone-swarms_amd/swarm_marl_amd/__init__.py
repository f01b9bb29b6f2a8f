"""swarm_marl_amd — MI355X-native vectorised drone-swarm step/observe/reward engine.

Host side of the C-ABI in include/swarm_mi355x.h.  `VecSwarm` is the batched tensor API;
`envs` holds the reference-compatible RLlib / Gymnasium classes.
"""
from .envs.common import DroneEnvConfig
from .vec_env import VecSwarm

__all__ = ["DroneEnvConfig", "VecSwarm"]
__version__ = "0.1.0"
