"""GPU: the config-5 specialisation swarm_step256w (N = 256, K = 3, Ms = 4, 4 <= M <= 16, kinematic;
one env per 512-thread workgroup, every pair evaluated once, two waves per 64-drone block) against the generic block-team kernel
swarm_kernel<0, 0, 4, 5, 0> (kernel_path="generic") on identical inputs — observations, flags,
infos, global state and every state tensor bit-identical, rewards within the 1e-5 contract (the
formation partial sums are added in a different order) — step after step with in-kernel
auto-reset, with inactive agents (the masked formation / minimum pass), clustered swarms (pair
collisions, the exact band, near-ties and the general finish) and against the CPU oracle.  The
N = 256 cases of test_gpu_parity.py / test_gpu_configs.py run through step256 as well.
Reference: src/swarm_marl/envs/drone_swarm_env.py:92-291.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from tests.helpers import oracle_cfg, vec_state_numpy

pytestmark = pytest.mark.gpu
REWARD_TOL = 1e-5
N = 256


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _pair(dev, raw, e, **kw):
    from swarm_marl_amd import VecSwarm
    kw.setdefault("with_infos", True)
    kw.setdefault("with_global_state", True)
    a = VecSwarm(e, raw, device=dev, kernel_path="auto", **kw)
    b = VecSwarm(e, raw, device=dev, kernel_path="generic", **kw)
    return a, b


EXACT = ("obs", "terminated", "truncated", "env_done", "dist_goal", "info_flags", "global_state",
         "pos", "vel", "goal", "obstacles", "active", "step_count", "episode")


def _assert_same(a, b, tag):
    for name in EXACT:
        x, y = getattr(a, name), getattr(b, name)
        if not torch.equal(x, y):
            bad = (x != y).nonzero()[:5].tolist()
            raise AssertionError(f"{tag}: {name} differs at {bad}")
    err = (a.reward.double() - b.reward.double()).abs().max().item()
    assert err <= REWARD_TOL, f"{tag}: reward err {err}"


def test_kernel_selection(dev):
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd import _native as nat
    v = VecSwarm(4, {"num_drones": N}, device=dev)
    assert int(v.launch_info.kernel_id) == nat.KERNEL_STEP256 and v.kernel_name() == "swarm_step256w"
    for raw in ({"num_drones": 255}, {"num_drones": N, "neighbor_k": 4}, {"num_drones": N, "sensed_obstacles": 3},
                {"num_drones": N, "num_obstacles": 3}, {"num_drones": N, "num_obstacles": 17}):
        assert int(VecSwarm(2, raw, device=dev).launch_info.kernel_id) == nat.KERNEL_GENERIC, raw
    assert int(VecSwarm(2, {"num_drones": N}, device=dev, dynamics="physics").launch_info.kernel_id) == \
        nat.KERNEL_GENERIC
    assert VecSwarm(2, {"num_drones": N}, device=dev, kernel_path="generic").kernel_name().startswith(
        "swarm_kernel<0, 0, 4, 5, 0>")


@pytest.mark.parametrize("m,max_steps,masked,radii", [(8, 9, False, None), (8, 400, True, None), (4, 6, False, 0.0),
                                                      (16, 12, True, None), (11, 5, False, 0.2)])
def test_step256_matches_generic_autoreset(dev, m, max_steps, masked, radii):
    raw = dict(num_drones=N, num_obstacles=m, max_steps=max_steps)
    if radii is not None:  # small / zero radii: continuing envs (the keys pass on the current positions)
        raw.update(collision_radius=radii, goal_radius=radii, obstacle_radius=radii)
    e = 96
    a, b = _pair(dev, raw, e, auto_reset=True, seed=5, env_offset=3)
    assert a.kernel_name() == "swarm_step256w"
    a.reset()
    b.reset()
    _assert_same(a, b, "reset")
    g = torch.Generator(device=dev).manual_seed(77 + m)
    resets = conts = 0
    for t in range(10):
        act = torch.rand((e, N, 3), device=dev, generator=g) * 2.6 - 1.3
        am = (torch.rand((e, N), device=dev, generator=g) > 0.1) if masked else None
        a.step(act, am)
        b.step(act, am)
        _assert_same(a, b, f"M={m} t={t}")
        done = (a.env_done & 4) != 0
        resets += int(done.sum())
        conts += int((~done).sum())
    assert resets > 0  # the reset's keys pass ran
    if radii is not None:
        assert conts > 0  # the continuing envs' keys pass ran (default radii: every env resets)


def test_step256_partial_activity(dev):
    """Inactive (removed) agents: the masked formation / minimum pass and the banded collision
    test; an env with every agent inactive exercises the n_active == 0 branch."""
    raw = dict(num_drones=N, collision_radius=0.3, goal_radius=0.5, obstacle_radius=0.3)
    e = 64
    a, b = _pair(dev, raw, e, auto_reset=False, seed=1)
    a.reset()
    b.reset()
    gen = torch.Generator(device=dev).manual_seed(3)
    active = torch.rand((e, N), device=dev, generator=gen) > 0.3
    active[0] = False
    active[1] = True
    active[2, 1:] = False
    for v in (a, b):
        v.set_state(active=active)
    for t in range(6):
        act = torch.rand((e, N, 3), device=dev, generator=gen) * 2 - 1
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"partial t={t}")


def test_step256_dense_clusters(dev):
    """Clustered swarms: pair collisions inside and near the exact band, lattice duplicates and
    coincident drones (key near-ties, the general finish and exact selection)."""
    raw = dict(num_drones=N, max_steps=50)
    e = 48
    a, b = _pair(dev, raw, e, auto_reset=True, seed=9)
    gen = torch.Generator(device="cpu").manual_seed(4)
    centre = torch.rand((e, 1, 3), generator=gen) * 16 - 8
    spread = torch.linspace(0.5, 6.0, e).view(e, 1, 1)
    pos = (centre + torch.randn((e, N, 3), generator=gen) * spread).clamp(-10, 10)
    pos[::5] = torch.round(pos[::5])  # lattice-like duplicates and exact ties
    pos[1::9, 128:] = pos[1::9, :128]  # coincident pairs across waves
    obst = torch.rand((e, 8, 3), generator=gen) * 20 - 10
    obst[::3, 4:] = obst[::3, :4]      # duplicated obstacles: obstacle near-ties
    for v in (a, b):
        v.set_state(pos=pos, vel=torch.zeros_like(pos), goal=torch.zeros((e, 3)), obstacles=obst,
                    active=torch.ones((e, N), dtype=torch.bool))
    for t in range(3):
        act = torch.zeros((e, N, 3), device=dev)
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"cluster t={t}")


def test_step256_vs_oracle(dev):
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    raw = dict(num_drones=N, max_steps=5)
    cfg = oracle_cfg(raw)
    e = 6
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=21, with_infos=True, with_global_state=True)
    assert vec.kernel_name() == "swarm_step256w"
    vec.reset()
    torch.cuda.synchronize()
    st = vec_state_numpy(vec)
    rng = np.random.default_rng(8)
    for t in range(6):
        act = rng.uniform(-1.2, 1.2, (e, N, 3)).astype(np.float32)
        am = rng.uniform(size=(e, N)) > 0.2
        vec.step(torch.as_tensor(act).to(dev), torch.as_tensor(am).to(dev))
        torch.cuda.synchronize()
        st, out = so.step(cfg, st, act, am, auto_reset=True, seed=21, exact_formation=False)
        assert np.array_equal(vec.obs.cpu().numpy(), out["obs"]), f"obs t={t}"
        err = np.abs(vec.reward.cpu().numpy().astype(np.float64) - out["reward"]).max()
        assert err <= REWARD_TOL, f"reward err {err} t={t}"
        assert np.array_equal(vec.terminated.cpu().numpy(), out["terminated"])
        assert np.array_equal(vec.truncated.cpu().numpy(), out["truncated"])
        assert np.array_equal((vec.env_done.cpu().numpy() & 4) != 0, out["reset"])
        got = vec_state_numpy(vec)
        for k in ("pos", "vel", "goal", "obst", "active", "step", "episode"):
            assert np.array_equal(got[k], st[k]), f"state {k} t={t}"
        assert np.array_equal(vec.global_state.cpu().numpy(), out["global_state"])


@pytest.mark.parametrize("e,groups", [(1, 1), (1030, 3)])
def test_step256_single_env_and_groups(dev, e, groups):
    """One env (one 512-thread workgroup), and a batch split into env groups of unequal size on
    their own streams (swarm_step_groups) — against the generic kernel step after step."""
    raw = dict(num_drones=N, max_steps=7)
    a, b = _pair(dev, raw, e, auto_reset=True, seed=13, groups=groups)
    assert a.kernel_name() == "swarm_step256w"
    a.reset()
    b.reset()
    g = torch.Generator(device=dev).manual_seed(19)
    for t in range(3):
        act = torch.rand((e, N, 3), device=dev, generator=g) * 2 - 1
        a.step(act)
        b.step(act)
        torch.cuda.synchronize()
        _assert_same(a, b, f"E={e} groups={groups} t={t}")
