"""ctypes binding of the C-ABI in include/swarm_mi355x.h (libswarm_mi355x.so, built for gfx950).

The library is the product's compute path: there is no CPU fallback.  If it is missing the
import of the engine fails loudly (NativeLibraryError) — build it with
`python -c "import __graft_entry__ as g; g.build()"` from the repository root.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_NAME = "libswarm_mi355x.so"
LIB_DIR = Path(__file__).resolve().parent / "_lib"
LIB_PATH = LIB_DIR / LIB_NAME

ABI_VERSION = 5
WORK_WORDS = 256  # SWARM_WORK_WORDS: u32 env-queue heads of the persistent swarm_step64

PATH_AUTO = 0
PATH_GENERIC = 1
KERNEL_GENERIC = 0
KERNEL_STEP64 = 1
KERNEL_STEP64_PERSISTENT = 2
KERNEL_STEP16Q = 3
KERNEL_STEP256 = 4

SWARM_OK = 0
SWARM_EINVAL = -1
SWARM_ENULL = -2
SWARM_ELIMIT = -3
SWARM_EHIP = -4

DYN_KINEMATIC = 0
DYN_POINTMASS_PHYSICS = 1
REW_SWARM = 0
REW_PHYSICS = 1

ENV_TERMINATED = 1
ENV_TRUNCATED = 2
ENV_RESET = 4

AGENT_STEPPED = 1
AGENT_REACHED = 2
AGENT_COLLISION = 4
AGENT_HAS_OBS = 8

POLICY_HIDDEN = 256
POLICY_MAX_IN = 47
POLICY_MAX_OUT = 12
POLICY_BF16 = 0
POLICY_F32 = 1
POLICY_F32X3 = 2
POLICY_ACT_MEAN = 0
POLICY_ACT_SAMPLE = 1
EVAL_LIVE = 1
EVAL_COLLIDED = 2
EVAL_STEP_FUSED = 1
EVAL_RECORD = 9
EVAL_SEGMENTS = 64

# every symbol include/swarm_mi355x.h declares
EXPORTED_SYMBOLS = (
    "swarm_abi_version", "swarm_last_error", "swarm_params_default", "swarm_obs_dim",
    "swarm_query_launch", "swarm_step", "swarm_step_groups", "swarm_reset", "swarm_observe",
    "swarm_policy_packed_bytes", "swarm_policy_pack", "swarm_policy_forward", "swarm_policy_last_error",
    "swarm_eval_begin", "swarm_eval_update", "swarm_eval_single_update", "swarm_eval_last_error",
    "swarm_env_cfg_set",
)
ENV_CFG_BYTES = 64  # sizeof(swarm_env_cfg_t)


class NativeLibraryError(RuntimeError):
    pass


class SwarmParams(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("num_envs", ctypes.c_int32),
        ("num_drones", ctypes.c_int32),
        ("num_obstacles", ctypes.c_int32),
        ("sensed_obstacles", ctypes.c_int32),
        ("neighbor_k", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("dynamics", ctypes.c_int32),
        ("reward_mode", ctypes.c_int32),
        ("auto_reset", ctypes.c_int32),
        ("physics_substeps", ctypes.c_int32),
        ("damping_law", ctypes.c_int32),
        ("env_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("world_size", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("max_speed", ctypes.c_double),
        ("max_accel", ctypes.c_double),
        ("collision_radius", ctypes.c_double),
        ("goal_radius", ctypes.c_double),
        ("obstacle_radius", ctypes.c_double),
        ("desired_spacing", ctypes.c_double),
        ("reward_progress_scale", ctypes.c_double),
        ("reward_goal", ctypes.c_double),
        ("reward_collision", ctypes.c_double),
        ("reward_formation_scale", ctypes.c_double),
        ("gravity", ctypes.c_double),
        ("gravity_comp", ctypes.c_double),
        ("substep_dt", ctypes.c_double),
        ("drone_contact_radius", ctypes.c_double),
        ("ground_contact_height", ctypes.c_double),
        ("kernel_path", ctypes.c_int32),
        ("waves_per_simd", ctypes.c_int32),
    ]


class SwarmState(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("pos", "vel", "goal", "obstacles", "active", "step_count", "episode", "damping",
                 "work", "env_cfg", "env_cfg_next")]


class SwarmEnvCfg(ctypes.Structure):
    """swarm_env_cfg_t: one env's derived parameters (64 B)."""
    _fields_ = [(name, ctypes.c_float) for name in
                ("half_w", "neg_half_w", "width_w", "dt", "max_speed", "max_accel", "s_vmax", "s_obst",
                 "s_phys_obst")] + [("max_steps", ctypes.c_int32), ("num_obstacles", ctypes.c_int32),
                                    ("reserved", ctypes.c_int32), ("max_speed_d", ctypes.c_double),
                                    ("world_size", ctypes.c_double)]


ENV_OVERRIDE_FIELDS = ("world_size", "dt", "max_speed", "max_accel", "obstacle_radius", "max_steps",
                       "num_obstacles")


class SwarmEnvOverrides(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in ENV_OVERRIDE_FIELDS]


class SwarmOut(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("obs", "reward", "terminated", "truncated", "env_done", "dist_goal",
                 "info_flags", "global_state", "eval")]  # eval: host pointer to a SwarmEval (fused)


class SwarmPolicy(ctypes.Structure):
    _fields_ = [("in_dim", ctypes.c_int32), ("out_dim", ctypes.c_int32), ("precision", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("weights", ctypes.c_void_p)]


class SwarmEval(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("ep_reward", "ep_steps", "reached_step", "status", "fe_sum", "start", "goal", "last",
                 "traveled", "records", "count")] + [("capacity", ctypes.c_int32), ("update_index", ctypes.c_int32),
                                                     ("flags", ctypes.c_int32), ("seg_base", ctypes.c_int32),
                                                     ("segments", ctypes.c_int32),
                                                     ("state_pos", ctypes.c_void_p), ("state_goal", ctypes.c_void_p)]


class SwarmLaunchInfo(ctypes.Structure):
    _fields_ = [(name, ctypes.c_int32) for name in
                ("threads_per_block", "envs_per_block", "lanes_per_env", "blocks", "lds_bytes",
                 "neighbor_slots", "obstacle_slots", "obs_dim", "staged_obs", "kernel_id")]


_LIB = None


def load_library(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load libswarm_mi355x.so (once) and declare its signatures."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    if path is None and os.environ.get("SWARM_MI355X_LIB"):
        path = os.environ["SWARM_MI355X_LIB"]  # diagnostic builds (tools/ablate.sh)
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise NativeLibraryError(
            f"{p} is missing: the MI355X swarm engine has no CPU fallback. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` in the repository root.")
    lib = ctypes.CDLL(str(p))
    P, S, O = ctypes.POINTER(SwarmParams), ctypes.POINTER(SwarmState), ctypes.POINTER(SwarmOut)
    vp = ctypes.c_void_p
    lib.swarm_abi_version.restype = ctypes.c_int
    lib.swarm_abi_version.argtypes = []
    lib.swarm_last_error.restype = ctypes.c_char_p
    lib.swarm_last_error.argtypes = []
    lib.swarm_params_default.restype = None
    lib.swarm_params_default.argtypes = [P]
    lib.swarm_obs_dim.restype = ctypes.c_int
    lib.swarm_obs_dim.argtypes = [P]
    lib.swarm_query_launch.restype = ctypes.c_int
    lib.swarm_query_launch.argtypes = [P, ctypes.POINTER(SwarmLaunchInfo)]
    lib.swarm_step.restype = ctypes.c_int
    lib.swarm_step.argtypes = [P, S, vp, vp, O, vp]
    lib.swarm_step_groups.restype = ctypes.c_int
    lib.swarm_step_groups.argtypes = [P, S, vp, vp, O, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                      ctypes.POINTER(ctypes.c_void_p)]
    lib.swarm_reset.restype = ctypes.c_int
    lib.swarm_reset.argtypes = [P, S, vp, O, vp]
    lib.swarm_observe.restype = ctypes.c_int
    lib.swarm_observe.argtypes = [P, S, vp, O, vp]
    fp = ctypes.POINTER(ctypes.c_float)
    lib.swarm_policy_packed_bytes.restype = ctypes.c_longlong
    lib.swarm_policy_packed_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.swarm_policy_pack.restype = ctypes.c_int
    lib.swarm_policy_pack.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, fp, fp, fp, fp, fp, fp, vp]
    lib.swarm_policy_forward.restype = ctypes.c_int
    lib.swarm_policy_forward.argtypes = [ctypes.POINTER(SwarmPolicy), vp, ctypes.c_longlong, vp, vp, ctypes.c_int,
                                         ctypes.c_ulonglong, ctypes.c_ulonglong, vp]
    lib.swarm_policy_last_error.restype = ctypes.c_char_p
    lib.swarm_policy_last_error.argtypes = []
    ev = ctypes.POINTER(SwarmEval)
    lib.swarm_eval_begin.restype = ctypes.c_int
    lib.swarm_eval_begin.argtypes = [P, ev, O, vp, vp]
    lib.swarm_eval_update.restype = ctypes.c_int
    lib.swarm_eval_update.argtypes = [P, ev, O, vp]
    lib.swarm_eval_single_update.restype = ctypes.c_int
    lib.swarm_eval_single_update.argtypes = [P, ev, O, vp, vp]
    lib.swarm_eval_last_error.restype = ctypes.c_char_p
    lib.swarm_eval_last_error.argtypes = []
    lib.swarm_env_cfg_set.restype = ctypes.c_int
    lib.swarm_env_cfg_set.argtypes = [P, ctypes.POINTER(SwarmEnvOverrides), vp, vp, vp]
    got = lib.swarm_abi_version()
    if got != ABI_VERSION:
        raise NativeLibraryError(f"{p}: ABI version {got}, expected {ABI_VERSION}")
    if path is None:
        _LIB = lib
    return lib


def check(rc: int, lib: ctypes.CDLL | None = None, policy: bool = False, which: str | None = None) -> None:
    """Raise on a negative return code (bad arguments -> ValueError, HIP errors -> RuntimeError).
    `which` names the component whose last-error string explains it ("policy", "eval")."""
    if rc == SWARM_OK:
        return
    lib = lib or load_library()
    which = "policy" if policy else which
    err = {"policy": lib.swarm_policy_last_error, "eval": lib.swarm_eval_last_error}.get(which, lib.swarm_last_error)
    msg = (err() or b"").decode(errors="replace")
    if rc in (SWARM_EINVAL, SWARM_ENULL, SWARM_ELIMIT):
        raise ValueError(f"swarm_mi355x error {rc}: {msg}")
    raise RuntimeError(f"swarm_mi355x error {rc}: {msg}")
