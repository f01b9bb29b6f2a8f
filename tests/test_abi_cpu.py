"""CPU: the C-ABI library (libswarm_mi355x.so) loads, exports exactly what include/swarm_mi355x.h
declares, and validates its arguments.  No kernel is launched: every call here either returns
before touching the GPU (validation, zero envs) or is a pure host query.
"""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "swarm_mi355x.h"


@pytest.fixture(scope="module")
def nat():
    from swarm_marl_amd import _native
    return _native


@pytest.fixture(scope="module")
def lib(nat):
    return nat.load_library()


def _declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|long long|const char\*)\s+(swarm_\w+)\s*\(", text, re.M)))


def test_header_symbols_are_exported(nat, lib):
    declared = _declared()
    assert declared == sorted(nat.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(nat.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(declared) <= exported
    # nothing else of ours leaks out of the shared object
    assert {s for s in exported if s.startswith("swarm_")} == set(declared)


def test_library_is_built_for_gfx950(nat):
    data = nat.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle id of the device code
    assert b"amdgcn-amd-amdhsa--gfx942" not in data  # MI355X only: no other device targets


def _params(nat, lib, **kw):
    p = nat.SwarmParams()
    lib.swarm_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def test_abi_version_and_defaults(nat, lib):
    from swarm_marl_amd.envs.common import DroneEnvConfig
    assert lib.swarm_abi_version() == nat.ABI_VERSION == 5
    p = _params(nat, lib)
    c = DroneEnvConfig()
    for name in ("max_steps", "num_obstacles", "sensed_obstacles", "neighbor_k"):
        assert getattr(p, name) == getattr(c, name), name
    for name in ("world_size", "dt", "max_speed", "max_accel", "collision_radius", "goal_radius",
                 "obstacle_radius", "desired_spacing", "reward_progress_scale", "reward_goal",
                 "reward_collision", "reward_formation_scale"):
        assert getattr(p, name) == getattr(c, name), name
    assert p.num_drones == 3 and p.dynamics == nat.DYN_KINEMATIC and p.auto_reset == 0


@pytest.mark.parametrize("k,ms", [(3, 4), (0, 0), (16, 16), (5, 2)])
def test_obs_dim(nat, lib, k, ms):
    p = _params(nat, lib, neighbor_k=k, sensed_obstacles=ms)
    assert lib.swarm_obs_dim(ctypes.byref(p)) == 9 + 4 * k + 4 * ms


@pytest.mark.parametrize("n", [1, 2, 3, 16, 33, 63, 64, 65, 100, 256, 1024])
def test_launch_geometry(nat, lib, n):
    p = _params(nat, lib, num_drones=n, num_envs=1000)
    info = nat.SwarmLaunchInfo()
    assert lib.swarm_query_launch(ctypes.byref(p), ctypes.byref(info)) == 0
    lanes = 1 << (n - 1).bit_length()
    if info.kernel_id == nat.KERNEL_STEP16Q:  # config-2 specialisation: 4 lanes per drone; one env per
        # 3-wave workgroup (rewards, observation, next episode)
        assert n == 16 and info.lanes_per_env == 64 and info.staged_obs == 0
        assert info.threads_per_block == 192 and info.envs_per_block == 1
        assert info.blocks == 1000 and 0 < info.lds_bytes <= 160 * 1024
        return
    if info.kernel_id == nat.KERNEL_STEP256:  # config-5 specialisation: one env per 512-thread workgroup
        # (two waves per 64-drone block: swarm_step256w), one lane per drone in each half
        assert n == 256 and info.lanes_per_env == 256 and info.staged_obs == 0
        assert info.threads_per_block == 512 and info.envs_per_block == 1
        assert info.blocks == 1000 and 0 < info.lds_bytes <= 64 * 1024
        return
    assert info.lanes_per_env == lanes
    if info.kernel_id == nat.KERNEL_STEP64:  # headline specialisation: 4 one-env waves per workgroup
        assert info.threads_per_block == 256 and info.envs_per_block == 4
    elif lanes <= 64:  # wave teams: 64/L envs per 64-thread workgroup
        assert info.threads_per_block == 64 and info.envs_per_block == 64 // lanes
    else:  # one env per workgroup of L threads
        assert info.threads_per_block == lanes and info.envs_per_block == 1
    assert info.blocks == -(-1000 // info.envs_per_block)
    assert 0 < info.lds_bytes <= 160 * 1024
    assert info.neighbor_slots == 4 and info.obstacle_slots == 5  # K=3 -> 4 keys, Ms=4 -> 5
    assert info.obs_dim == 37
    # obs rows from registers only for small launches of multi-team waves / block teams
    assert info.staged_obs == (1 if lanes == 64 or info.blocks > 2048 else 0)


def test_obs_direct_threshold(nat, lib):
    info = nat.SwarmLaunchInfo()
    # (N = 16 / 256 with the default K / Ms / M run swarm_step16q / swarm_step256w, rows from
    # registers at any E: the generic kernel's threshold is checked there with K = 4)
    for n, e, staged, extra in [(16, 1024, 0, {}), (16, 32768, 0, {}), (16, 1024, 0, {"neighbor_k": 4}),
                                (16, 8192, 0, {"neighbor_k": 4}), (16, 8193, 1, {"neighbor_k": 4}),
                                (16, 32768, 1, {"neighbor_k": 4}), (256, 1024, 0, {"neighbor_k": 4}),
                                (256, 4096, 1, {"neighbor_k": 4}), (256, 4096, 0, {}), (64, 1024, 1, {}),
                                (3, 4, 0, {})]:
        p = _params(nat, lib, num_drones=n, num_envs=e, **extra)
        assert lib.swarm_query_launch(ctypes.byref(p), ctypes.byref(info)) == 0
        assert info.staged_obs == staged, (n, e)


@pytest.mark.parametrize("field,value,code", [
    ("abi_version", 1, "EINVAL"), ("num_envs", -1, "EINVAL"), ("num_drones", 0, "ELIMIT"),
    ("num_drones", 1025, "ELIMIT"), ("neighbor_k", 17, "ELIMIT"), ("sensed_obstacles", 17, "ELIMIT"),
    ("num_obstacles", -2, "EINVAL"), ("dynamics", 7, "EINVAL"), ("reward_mode", 1, "EINVAL"),
    ("damping_law", 3, "EINVAL"), ("kernel_path", 2, "EINVAL"), ("waves_per_simd", 9, "EINVAL"),
    ("waves_per_simd", -1, "EINVAL"),
])
def test_validation_errors(nat, lib, field, value, code):
    kw = {field: value}
    if field == "sensed_obstacles":
        kw["num_obstacles"] = 20
    p = _params(nat, lib, **kw)
    info = nat.SwarmLaunchInfo()
    rc = lib.swarm_query_launch(ctypes.byref(p), ctypes.byref(info))
    assert rc == getattr(nat, "SWARM_" + code)
    assert lib.swarm_last_error()  # a message is set
    with pytest.raises(ValueError):
        nat.check(rc, lib)


def test_null_arguments_and_empty_batch(nat, lib):
    p = _params(nat, lib, num_envs=0)
    s, o = nat.SwarmState(), nat.SwarmOut()
    assert lib.swarm_step(None, ctypes.byref(s), None, None, ctypes.byref(o), None) == nat.SWARM_ENULL
    assert lib.swarm_step(ctypes.byref(p), None, None, None, ctypes.byref(o), None) == nat.SWARM_ENULL
    assert lib.swarm_query_launch(ctypes.byref(p), None) == nat.SWARM_ENULL
    # zero envs: a valid no-op (returns before any launch)
    assert lib.swarm_step(ctypes.byref(p), ctypes.byref(s), None, None, ctypes.byref(o), None) == 0
    assert lib.swarm_reset(ctypes.byref(p), ctypes.byref(s), None, ctypes.byref(o), None) == 0
    assert lib.swarm_observe(ctypes.byref(p), ctypes.byref(s), None, ctypes.byref(o), None) == 0
    # non-empty batch with missing buffers: rejected before any launch
    p2 = _params(nat, lib, num_envs=4)
    assert lib.swarm_step(ctypes.byref(p2), ctypes.byref(s), None, None, ctypes.byref(o), None) == nat.SWARM_ENULL
    assert b"NULL" in lib.swarm_last_error()


def test_missing_library_fails_loudly(nat, tmp_path):
    with pytest.raises(nat.NativeLibraryError):
        nat.load_library(tmp_path / "libswarm_mi355x.so")


def test_env_cfg_layout_matches_header(nat, tmp_path):
    """ctypes mirrors of the per-env records agree with the C compiler's layout of the header."""
    fields = [f for f, _ in nat.SwarmEnvCfg._fields_]
    src = tmp_path / "layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "swarm_mi355x.h"', "int main(void) {",
             'printf("%zu %zu %zu\\n", sizeof(swarm_env_cfg_t), sizeof(swarm_state_t), sizeof(swarm_env_overrides_t));']
    lines += [f'printf("%zu\\n", offsetof(swarm_env_cfg_t, {f}));' for f in fields]
    lines += [f'printf("%zu\\n", offsetof(swarm_state_t, {f}));' for f, _ in nat.SwarmState._fields_]
    lines += ["return 0; }"]
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    sizes, rest = [int(x) for x in out[:3]], [int(x) for x in out[3:]]
    assert sizes == [ctypes.sizeof(nat.SwarmEnvCfg), ctypes.sizeof(nat.SwarmState),
                     ctypes.sizeof(nat.SwarmEnvOverrides)]
    assert sizes[0] == nat.ENV_CFG_BYTES == 64
    assert rest[:len(fields)] == [getattr(nat.SwarmEnvCfg, f).offset for f in fields]
    assert rest[len(fields):] == [getattr(nat.SwarmState, f).offset for f, _ in nat.SwarmState._fields_]


def test_env_cfg_set_validation(nat, lib):
    ov = nat.SwarmEnvOverrides()
    p0 = _params(nat, lib, num_envs=0)
    assert lib.swarm_env_cfg_set(ctypes.byref(p0), ctypes.byref(ov), None, None, None) == 0  # empty: no-op
    p = _params(nat, lib, num_envs=4)
    assert lib.swarm_env_cfg_set(ctypes.byref(p), None, None, None, None) == nat.SWARM_ENULL
    assert lib.swarm_env_cfg_set(ctypes.byref(p), ctypes.byref(ov), None, None, None) == nat.SWARM_ENULL
    assert lib.swarm_env_cfg_set(ctypes.byref(_params(nat, lib, num_envs=4, num_drones=0)), ctypes.byref(ov),
                                 None, None, None) == nat.SWARM_ELIMIT
    # a next-episode record without a current one is rejected before any launch
    s, o = nat.SwarmState(), nat.SwarmOut()
    for name in ("pos", "vel", "goal", "obstacles", "active", "step_count", "episode"):
        setattr(s, name, 16)
    o.obs, o.reward, o.terminated, o.truncated, o.env_done = 16, 16, 16, 16, 16
    s.env_cfg_next = 64
    assert lib.swarm_step(ctypes.byref(p), ctypes.byref(s), 16, None, ctypes.byref(o), None) == nat.SWARM_ENULL
    assert b"env_cfg" in lib.swarm_last_error()


def test_step_groups_validation(nat, lib):
    """swarm_step_groups checks the params, the group split and its arrays before any launch."""
    s, o = nat.SwarmState(), nat.SwarmOut()
    envs = (ctypes.c_int32 * 3)(2, 1, 1)
    streams = (ctypes.c_void_p * 3)()
    p = _params(nat, lib, num_envs=4)
    args = (ctypes.byref(s), None, None, ctypes.byref(o))
    assert lib.swarm_step_groups(None, *args, 3, envs, streams) == nat.SWARM_ENULL
    assert lib.swarm_step_groups(ctypes.byref(p), None, None, None, ctypes.byref(o), 3, envs, streams) == nat.SWARM_ENULL
    assert lib.swarm_step_groups(ctypes.byref(p), *args, 0, envs, streams) == nat.SWARM_EINVAL
    assert lib.swarm_step_groups(ctypes.byref(p), *args, 3, None, streams) == nat.SWARM_ENULL
    assert lib.swarm_step_groups(ctypes.byref(p), *args, 3, envs, None) == nat.SWARM_ENULL
    assert lib.swarm_step_groups(ctypes.byref(p), *args, 2, envs, streams) == nat.SWARM_EINVAL  # 3 != 4 envs
    assert b"sum" in lib.swarm_last_error()
    neg = (ctypes.c_int32 * 3)(5, -1, 0)
    assert lib.swarm_step_groups(ctypes.byref(p), *args, 3, neg, streams) == nat.SWARM_EINVAL
    bad = _params(nat, lib, num_envs=4, num_drones=0)
    assert lib.swarm_step_groups(ctypes.byref(bad), *args, 3, envs, streams) == nat.SWARM_ELIMIT
    # the split is valid, the buffers are not: the first group's launch rejects them
    assert lib.swarm_step_groups(ctypes.byref(p), *args, 3, envs, streams) == nat.SWARM_ENULL
    # zero envs in every group: a valid no-op
    p0 = _params(nat, lib, num_envs=0)
    zero = (ctypes.c_int32 * 2)(0, 0)
    assert lib.swarm_step_groups(ctypes.byref(p0), *args, 2, zero, streams) == 0


@pytest.mark.parametrize("ctype,cname", [("SwarmOut", "swarm_out_t"), ("SwarmEval", "swarm_eval_t"),
                                         ("SwarmParams", "swarm_params_t"), ("SwarmPolicy", "swarm_policy_t"),
                                         ("SwarmLaunchInfo", "swarm_launch_info_t")])
def test_struct_layouts_match_header(nat, tmp_path, ctype, cname):
    """Every ctypes mirror of a header struct has the C compiler's size and field offsets."""
    cls = getattr(nat, ctype)
    fields = [f for f, _ in cls._fields_]
    src = tmp_path / "layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "swarm_mi355x.h"', "int main(void) {",
             f'printf("%zu\\n", sizeof({cname}));']
    lines += [f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields]
    lines += ["return 0; }"]
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert out[0] == ctypes.sizeof(cls)
    assert out[1:] == [getattr(cls, f).offset for f in fields]
