"""GPU: the config-2 specialisation swarm_step16q (N = 16, K = 3, Ms = 4, 4 <= M <= 16, kinematic;
one env per wave, four lanes per drone) against the generic swarm_kernel<0, 0, 4, 5, 1>
(kernel_path="generic") on identical inputs — observations, flags, infos, global state and every
state tensor bit-identical, rewards within the 1e-5 contract (the formation partial sums are
added in a different order) — step after step with in-kernel auto-reset, with inactive agents,
clustered swarms, coincident drones, and against the CPU oracle.  The N = 16 golden-fixture
replays of test_gpu_parity.py run through step16q as well.
Reference: src/swarm_marl/envs/drone_swarm_env.py:92-291.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from tests.helpers import oracle_cfg, vec_state_numpy

pytestmark = pytest.mark.gpu
REWARD_TOL = 1e-5


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
    v = VecSwarm(8, {"num_drones": 16}, device=dev)
    assert int(v.launch_info.kernel_id) == nat.KERNEL_STEP16Q and v.kernel_name() == "swarm_step16q"
    for raw in ({"num_drones": 15}, {"num_drones": 16, "neighbor_k": 4}, {"num_drones": 16, "sensed_obstacles": 3},
                {"num_drones": 16, "num_obstacles": 3}, {"num_drones": 16, "num_obstacles": 17}):
        assert int(VecSwarm(4, raw, device=dev).launch_info.kernel_id) == nat.KERNEL_GENERIC, raw
    assert int(VecSwarm(4, {"num_drones": 16}, device=dev, dynamics="physics").launch_info.kernel_id) == \
        nat.KERNEL_GENERIC
    assert VecSwarm(4, {"num_drones": 16}, device=dev, kernel_path="generic").kernel_name().startswith(
        "swarm_kernel<0, 0, 4, 5, 1>")


@pytest.mark.parametrize("m,max_steps,masked", [(8, 9, False), (8, 400, True), (4, 6, False),
                                                (16, 12, True), (11, 5, False)])
def test_step16q_matches_generic_autoreset(dev, m, max_steps, masked):
    raw = dict(num_drones=16, num_obstacles=m, max_steps=max_steps)
    e = 1023  # ragged last workgroup
    a, b = _pair(dev, raw, e, auto_reset=True, seed=5, env_offset=3)
    assert a.kernel_name() == "swarm_step16q"
    a.reset()
    b.reset()
    _assert_same(a, b, "reset")
    g = torch.Generator(device=dev).manual_seed(77 + m)
    resets = 0
    for t in range(16):
        act = torch.rand((e, 16, 3), device=dev, generator=g) * 2.6 - 1.3
        am = (torch.rand((e, 16), device=dev, generator=g) > 0.1) if masked else None
        a.step(act, am)
        b.step(act, am)
        _assert_same(a, b, f"M={m} t={t}")
        resets += int(((a.env_done & 4) != 0).sum())
    assert resets > 0  # the in-kernel reset path ran


def test_step16q_partial_activity(dev):
    """Inactive (removed) agents: the masked pair pass and the banded collision test; an env with
    every agent inactive exercises the n_active == 0 branch."""
    raw = dict(num_drones=16, collision_radius=1.2, goal_radius=1.5)
    e = 512
    a, b = _pair(dev, raw, e, auto_reset=False, seed=1)
    a.reset()
    b.reset()
    gen = torch.Generator(device=dev).manual_seed(3)
    active = torch.rand((e, 16), device=dev, generator=gen) > 0.3
    active[0] = False
    active[1] = True
    active[2, 1:] = False
    for v in (a, b):
        v.set_state(active=active)
    for t in range(8):
        act = torch.rand((e, 16, 3), device=dev, generator=gen) * 2 - 1
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"partial t={t}")


def test_step16q_dense_clusters(dev):
    """Clustered swarms: pair collisions, near ties and the general-finish fallback."""
    raw = dict(num_drones=16, max_steps=50)
    e = 256
    a, b = _pair(dev, raw, e, auto_reset=True, seed=9)
    gen = torch.Generator(device="cpu").manual_seed(4)
    centre = torch.rand((e, 1, 3), generator=gen) * 16 - 8
    spread = torch.linspace(0.2, 3.0, e).view(e, 1, 1)
    pos = (centre + torch.randn((e, 16, 3), generator=gen) * spread).clamp(-10, 10)
    pos[::5] = torch.round(pos[::5])  # lattice-like duplicates and exact ties
    pos[1::9, 8:] = pos[1::9, :8]     # coincident pairs
    obst = torch.rand((e, 8, 3), generator=gen) * 20 - 10
    obst[::3, 4:] = obst[::3, :4]     # duplicated obstacles: obstacle near-ties
    for v in (a, b):
        v.set_state(pos=pos, vel=torch.zeros_like(pos), goal=torch.zeros((e, 3)), obstacles=obst,
                    active=torch.ones((e, 16), dtype=torch.bool))
    for t in range(4):
        act = torch.zeros((e, 16, 3), device=dev)
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"cluster t={t}")


def test_step16q_vs_oracle(dev):
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    raw = dict(num_drones=16, max_steps=6)
    cfg = oracle_cfg(raw)
    e = 96
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=21, with_infos=True, with_global_state=True)
    assert vec.kernel_name() == "swarm_step16q"
    vec.reset()
    torch.cuda.synchronize()
    st = vec_state_numpy(vec)
    rng = np.random.default_rng(8)
    for t in range(10):
        act = rng.uniform(-1.2, 1.2, (e, 16, 3)).astype(np.float32)
        am = rng.uniform(size=(e, 16)) > 0.2
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


@pytest.mark.parametrize("radius", [0.0, 0.5])
def test_step16q_coincident_drones_vs_oracle(dev, radius):
    """Drones stacked on a few points: nearest keys of value 0, exact ties ordered by index."""
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    raw = dict(num_drones=16, collision_radius=radius, goal_radius=radius, max_steps=50)
    cfg = oracle_cfg(raw)
    e = 24
    v = VecSwarm(e, raw, device=dev, auto_reset=True, seed=3)
    v.reset()
    st = vec_state_numpy(v)
    rng = np.random.default_rng(11)
    corners = np.array([[10, 10, 10], [-10, 10, 10], [10, -10, -10], [3.25, -1.5, 2.0]], np.float32)
    pos = st["pos"].copy()
    for k in range(e):
        pos[k] = corners[rng.integers(0, 1 + k % 4, 16)]
        pos[k, : k % 7] += rng.uniform(-3, 3, (k % 7, 3)).astype(np.float32)
    v.set_state(pos=pos, vel=np.zeros_like(pos), active=np.ones((e, 16), bool), step_count=np.zeros(e, np.int32))
    for t in range(3):
        st = vec_state_numpy(v)
        act = np.zeros((e, 16, 3), np.float32) if t == 0 else rng.uniform(-1, 1, (e, 16, 3)).astype(np.float32)
        v.step(torch.as_tensor(act, device=dev))
        ns, out = so.step(cfg, st, act, auto_reset=True, seed=3)
        assert np.array_equal(v.obs.cpu().numpy(), out["obs"]), f"t={t} obs"
        assert np.abs(v.reward.cpu().numpy().astype(np.float64) - out["reward"]).max() < REWARD_TOL, f"t={t}"
        assert np.array_equal(v.terminated.cpu().numpy(), out["terminated"]), f"t={t}"
        assert np.array_equal(vec_state_numpy(v)["pos"], ns["pos"]), f"t={t}"


@pytest.mark.parametrize("radius", [0.8, 0.5, 1.0 / 3.0])
def test_step16q_goal_radius_boundary(dev, radius):
    """step16q decides `reached` in squared space (s <= s_goal, the largest float s whose correctly
    rounded root is <= goal_radius) instead of comparing sqrt_rn(s) in f64: drones placed ulp by
    ulp across the goal radius must reach exactly as in the generic kernel."""
    raw = dict(num_drones=16, collision_radius=0.0, goal_radius=radius, max_steps=50)
    e = 8
    a, b = _pair(dev, raw, e, auto_reset=False, seed=2)
    a.reset()
    b.reset()
    x0 = np.float32(radius)
    xs = [x0]
    for _ in range(64):
        xs.insert(0, np.nextafter(xs[0], np.float32(0)))
        xs.append(np.nextafter(xs[-1], np.float32(10)))
    xs = np.array(xs[: e * 16], np.float32)  # 128 consecutive floats around the radius
    pos = np.zeros((e, 16, 3), np.float32)
    pos[:, :, 0] = xs.reshape(e, 16)
    obst = np.full((e, 8, 3), 9.0, np.float32)
    obst[:, :, 1] = np.linspace(-9, 9, 8, dtype=np.float32)
    for v in (a, b):
        v.set_state(pos=pos, vel=np.zeros_like(pos), goal=np.zeros((e, 3), np.float32), obstacles=obst,
                    active=np.ones((e, 16), bool), step_count=np.zeros(e, np.int32))
    act = torch.zeros((e, 16, 3), device=dev)
    a.step(act)
    b.step(act)
    _assert_same(a, b, f"goal boundary r={radius}")
    reached = (a.info_flags.cpu().numpy() & 2) != 0
    assert 0 < reached.sum() < reached.size  # the boundary runs through the sample


@pytest.mark.parametrize("e,groups", [(1, 1), (7, 1), (1001, 3)])
def test_step16q_xcd_order_ragged_and_groups(dev, e, groups):
    """The XCD-aware workgroup order (round 6: XCD x takes a contiguous block of envs) on grids that
    are not multiples of 8 and on env groups of unequal size launched on their own streams: every env
    is stepped exactly once, as by the generic kernel."""
    raw = dict(num_drones=16, max_steps=6)
    a, b = _pair(dev, raw, e, auto_reset=True, seed=23, groups=groups)
    assert a.kernel_name() == "swarm_step16q"
    a.reset()
    b.reset()
    g = torch.Generator(device=dev).manual_seed(29)
    for t in range(8):
        act = torch.rand((e, 16, 3), device=dev, generator=g) * 2 - 1
        a.step(act)
        b.step(act)
        torch.cuda.synchronize()
        _assert_same(a, b, f"E={e} groups={groups} t={t}")
