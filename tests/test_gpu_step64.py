"""GPU: the headline specialisation swarm_step64 (N = 64, K = 3, Ms = 4, 4 <= M <= 16, kinematic)
against the generic swarm_kernel (kernel_path="generic") on identical inputs — every output and
every state tensor bit-identical (kinematic rewards within 1e-5: the formation sum's f32 chain),
step after step with in-kernel auto-reset — and against the CPU oracle.  The golden-fixture / oracle tests of test_gpu_parity.py at N = 64 run through step64 too.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from tests.helpers import oracle_cfg, vec_state_numpy

pytestmark = pytest.mark.gpu


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


OUTS = ("obs", "terminated", "truncated", "env_done", "dist_goal", "info_flags", "global_state")
STATE = ("pos", "vel", "goal", "obstacles", "active", "step_count", "episode")
# round 6: step64 sums a pass's formation terms in one f32 chain (the generic kernel widens every
# 4-rotation group to f64), so kinematic rewards agree within the 1e-5 reward contract, not bit for
# bit; everything else (and the physics rewards, which carry no formation term) stays bitwise
REWARD_TOL = 1e-5


def _assert_same(a, b, tag, reward_exact=False):
    for name in OUTS + STATE:
        x, y = getattr(a, name), getattr(b, name)
        if not torch.equal(x, y):
            bad = (x != y).nonzero()[:5].tolist()
            raise AssertionError(f"{tag}: {name} differs at {bad}")
    if reward_exact:
        assert torch.equal(a.reward, b.reward), f"{tag}: reward differs"
    err = (a.reward.double() - b.reward.double()).abs().max().item()
    assert err <= REWARD_TOL, f"{tag}: reward err {err}"


def test_kernel_selection():
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd import _native as nat
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = torch.device("cuda", 0)
    assert VecSwarm(4, {"num_drones": 64}, device=d).kernel_name() == "swarm_step64_once<32, 4>"
    assert int(VecSwarm(4, {"num_drones": 64}, device=d).launch_info.kernel_id) == nat.KERNEL_STEP64
    for raw in ({"num_drones": 63}, {"num_drones": 64, "neighbor_k": 4},
                {"num_drones": 64, "sensed_obstacles": 3}, {"num_drones": 64, "num_obstacles": 3},
                {"num_drones": 64, "num_obstacles": 17}):
        v = VecSwarm(4, raw, device=d)
        assert int(v.launch_info.kernel_id) == nat.KERNEL_GENERIC, raw
    v = VecSwarm(4, {"num_drones": 64}, device=d, dynamics="physics")
    assert int(v.launch_info.kernel_id) == nat.KERNEL_STEP64
    assert v.kernel_name() == "swarm_step64_phys_once<32, 4>"
    v = VecSwarm(4, {"num_drones": 64}, device=d, dynamics="physics", waves_per_simd=4)
    assert int(v.launch_info.kernel_id) == nat.KERNEL_STEP64  # physics: one wave per env only
    v = VecSwarm(4, {"num_drones": 64}, device=d, kernel_path="generic")
    assert v.kernel_name().startswith("swarm_kernel<0, 0, 4, 5, 2>")


@pytest.mark.parametrize("m,max_steps,masked", [(8, 9, False), (8, 400, True), (4, 6, False),
                                                (16, 12, True), (11, 5, False)])
def test_step64_matches_generic_autoreset(dev, m, max_steps, masked):
    raw = dict(num_drones=64, num_obstacles=m, max_steps=max_steps)
    e = 2048
    a, b = _pair(dev, raw, e, auto_reset=True, seed=5, env_offset=3)
    assert a.kernel_name().startswith("swarm_step64")
    a.reset()
    b.reset()
    _assert_same(a, b, "reset")
    g = torch.Generator(device=dev).manual_seed(77 + m)
    resets = 0
    for t in range(14):
        act = torch.rand((e, 64, 3), device=dev, generator=g) * 2.6 - 1.3
        am = (torch.rand((e, 64), device=dev, generator=g) > 0.1) if masked else None
        a.step(act, am)
        b.step(act, am)
        _assert_same(a, b, f"M={m} t={t}")
        resets += int(((a.env_done & 4) != 0).sum())
    assert resets > 0  # the in-kernel reset path ran


def test_step64_partial_activity(dev):
    """Inactive (removed) agents put the wave on the masked pair pass and the banded collision
    test; an env with every agent inactive exercises the n_active == 0 branch."""
    raw = dict(num_drones=64, collision_radius=0.9)
    e = 512
    a, b = _pair(dev, raw, e, auto_reset=False, seed=1)
    a.reset()
    b.reset()
    gen = torch.Generator(device=dev).manual_seed(3)
    active = torch.rand((e, 64), device=dev, generator=gen) > 0.3
    active[0] = False
    active[1] = True
    active[2, 1:] = False
    for v in (a, b):
        v.set_state(active=active)
    for t in range(6):
        act = torch.rand((e, 64, 3), device=dev, generator=gen) * 2 - 1
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"partial t={t}")


def test_step64_dense_clusters(dev):
    """Clustered swarms: many pair collisions, near ties and exact-fallback selections."""
    raw = dict(num_drones=64, max_steps=50)
    e = 256
    a, b = _pair(dev, raw, e, auto_reset=True, seed=9)
    gen = torch.Generator(device="cpu").manual_seed(4)
    centre = torch.rand((e, 1, 3), generator=gen) * 16 - 8
    spread = torch.linspace(0.3, 3.0, e).view(e, 1, 1)
    pos = (centre + torch.randn((e, 64, 3), generator=gen) * spread).clamp(-10, 10)
    pos[::7] = torch.round(pos[::7])  # lattice-like duplicates and exact ties
    obst = torch.rand((e, 8, 3), generator=gen) * 20 - 10
    for v in (a, b):
        v.set_state(pos=pos, vel=torch.zeros_like(pos), goal=torch.zeros((e, 3)), obstacles=obst,
                    active=torch.ones((e, 64), dtype=torch.bool))
    for t in range(4):
        act = torch.zeros((e, 64, 3), device=dev)
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"cluster t={t}")


def test_step64_vs_oracle(dev):
    from oracle import swarm_oracle as so
    raw = dict(num_drones=64, max_steps=6)
    cfg = oracle_cfg(raw)
    e = 96
    from swarm_marl_amd import VecSwarm
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=21, with_infos=True,
                   with_global_state=True)
    assert vec.kernel_name().startswith("swarm_step64")
    vec.reset()
    torch.cuda.synchronize()
    st = vec_state_numpy(vec)
    rng = np.random.default_rng(8)
    for t in range(8):
        act = rng.uniform(-1.2, 1.2, (e, 64, 3)).astype(np.float32)
        am = rng.uniform(size=(e, 64)) > 0.2
        vec.step(torch.as_tensor(act).to(dev), torch.as_tensor(am).to(dev))
        torch.cuda.synchronize()
        st, out = so.step(cfg, st, act, am, auto_reset=True, seed=21, exact_formation=False)
        assert np.array_equal(vec.obs.cpu().numpy(), out["obs"]), f"obs t={t}"
        err = np.abs(vec.reward.cpu().numpy().astype(np.float64) - out["reward"]).max()
        assert err <= 1e-5, f"reward err {err} t={t}"
        assert np.array_equal(vec.terminated.cpu().numpy(), out["terminated"])
        assert np.array_equal(vec.truncated.cpu().numpy(), out["truncated"])
        ed = vec.env_done.cpu().numpy()
        assert np.array_equal((ed & 4) != 0, out["reset"])
        got = vec_state_numpy(vec)
        for k in ("pos", "vel", "goal", "obst", "active", "step", "episode"):
            assert np.array_equal(got[k], st[k]), f"state {k} t={t}"
        assert np.array_equal(vec.global_state.cpu().numpy(), out["global_state"])


@pytest.mark.parametrize("wps,e", [(1, 3000), (2, 2500)])
def test_step64_persistent_queue_matches_generic(dev, wps, e):
    """Persistent grid (fewer resident waves than envs): the per-XCD env queues hand out the
    rest.  Several launches in a row (each must leave the queue heads at zero) with in-kernel
    resets, bit-identical to the generic kernel; E not a multiple of 8 (ragged head ranges)."""
    raw = dict(num_drones=64, max_steps=5)
    a, b = _pair(dev, raw, e, auto_reset=True, seed=13, env_offset=5, waves_per_simd=wps)
    assert a.kernel_name() == "swarm_step64<32>"
    assert int(a.launch_info.blocks) < e
    a.reset()
    b.reset()
    g = torch.Generator(device=dev).manual_seed(99)
    for t in range(8):
        act = torch.rand((e, 64, 3), device=dev, generator=g) * 2 - 1
        a.step(act)
        b.step(act)
        _assert_same(a, b, f"persistent wps={wps} t={t}")
        assert int(torch.count_nonzero(a.work)) == 0, "queue heads not reset"


@pytest.mark.parametrize("m,max_steps,masked,law", [(8, 9, False, 0), (8, 400, True, 0), (4, 6, False, 1),
                                                    (16, 12, True, 1), (11, 5, False, 0)])
def test_step64_physics_matches_generic(dev, m, max_steps, masked, law):
    """swarm_step64_phys_once vs swarm_kernel<0, 1, 4, 5, 2>: bit-identical outputs and state
    (damping included) over steps with auto-resets, both damping laws, with / without masks."""
    raw = dict(num_drones=64, num_obstacles=m, max_steps=max_steps)
    e = 2048
    a, b = _pair(dev, raw, e, auto_reset=True, seed=9, env_offset=5, dynamics="physics",
                 physics={"damping_law": law})
    assert a.kernel_name() == "swarm_step64_phys_once<32, 4>"
    assert b.kernel_name().startswith("swarm_kernel<0, 1, 4, 5, 2>")
    a.reset()
    b.reset()
    _assert_same(a, b, "reset")
    g = torch.Generator(device=dev).manual_seed(91 + m)
    resets = 0
    for t in range(14):
        act = torch.rand((e, 64, 3), device=dev, generator=g) * 3.0 - 1.5
        am = (torch.rand((e, 64), device=dev, generator=g) > 0.1) if masked else None
        a.step(act, am)
        b.step(act, am)
        _assert_same(a, b, f"physics t={t}", reward_exact=True)
        assert torch.equal(a.damping, b.damping), f"physics t={t}: damping"
        resets += int(((a.env_done & 4) != 0).sum())
    assert resets > 0


def test_step64_physics_vs_oracle(dev):
    """A 32-env slice of the physics step64 batch against the oracle's point-mass restatement."""
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    raw = dict(num_drones=64, num_obstacles=8, max_steps=7)
    cfg = oracle_cfg(raw)
    e = 32
    v = VecSwarm(e, raw, device=dev, auto_reset=True, seed=13, dynamics="physics", with_infos=True,
                 with_global_state=True)
    assert v.kernel_name() == "swarm_step64_phys_once<32, 4>"
    v.reset()
    g = torch.Generator(device=dev).manual_seed(5)
    for t in range(9):
        st = vec_state_numpy(v)
        act = torch.rand((e, 64, 3), device=dev, generator=g) * 2 - 1
        v.step(act)
        ns, out = so.step(cfg, st, act.cpu().numpy(), physics=True, auto_reset=True, seed=13)
        assert np.array_equal(v.obs.cpu().numpy(), out["obs"]), f"t={t} obs"
        assert np.abs(v.reward.cpu().numpy().astype(np.float64) - out["reward"]).max() < 1e-5, f"t={t}"
        for k in ("pos", "vel", "goal", "obst", "active", "step", "episode", "damping"):
            assert np.array_equal(vec_state_numpy(v)[k], ns[k]), f"t={t} {k}"


@pytest.mark.parametrize("radius,dyn", [(0.0, "kinematic"), (0.5, "kinematic"), (0.0, "physics")])
@pytest.mark.parametrize("path", ["auto", "generic"])
def test_coincident_drones_vs_oracle(dev, radius, dyn, path):
    """Drones stacked on a few points (world-clip corners): nearest keys of value 0 decide the
    pair contact without the exact scan; obs (exact ties ordered by index), rewards and flags as
    the oracle, with zero and default radii."""
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    raw = dict(num_drones=64, collision_radius=radius, goal_radius=radius, max_steps=50)
    cfg = oracle_cfg(raw)
    e = 24
    v = VecSwarm(e, raw, device=dev, auto_reset=True, seed=3, dynamics=dyn, kernel_path=path)
    v.reset()
    st = vec_state_numpy(v)
    rng = np.random.default_rng(11)
    corners = np.array([[10, 10, 10], [-10, 10, 10], [10, -10, -10], [3.25, -1.5, 2.0]], np.float32)
    pos = st["pos"].copy()
    for k in range(e):
        ncorner = 1 + k % 4
        pos[k] = corners[rng.integers(0, ncorner, 64)]
        pos[k, : k % 7] += rng.uniform(-3, 3, (k % 7, 3)).astype(np.float32)
    v.set_state(pos=pos, vel=np.zeros_like(pos), active=np.ones((e, 64), bool),
                step_count=np.zeros(e, np.int32))
    for t in range(3):
        st = vec_state_numpy(v)
        act = np.zeros((e, 64, 3), np.float32) if t == 0 else rng.uniform(-1, 1, (e, 64, 3)).astype(np.float32)
        v.step(torch.as_tensor(act, device=dev))
        ns, out = so.step(cfg, st, act, physics=dyn == "physics", auto_reset=True, seed=3)
        assert np.array_equal(v.obs.cpu().numpy(), out["obs"]), f"t={t} obs"
        assert np.abs(v.reward.cpu().numpy().astype(np.float64) - out["reward"]).max() < 1e-5, f"t={t}"
        assert np.array_equal(v.terminated.cpu().numpy(), out["terminated"]), f"t={t}"
        assert np.array_equal(vec_state_numpy(v)["pos"], ns["pos"]), f"t={t}"
