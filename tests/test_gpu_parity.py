"""GPU parity: the HIP kernel (through the C-ABI) vs the reference fixtures and the CPU oracle.

Bar (BASELINE.json north_star): obs bit-exact, state/flags exact, rewards within 1e-5 absolute
(float32 reward output vs the reference's float64).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from tests.helpers import ROLLOUT_FIXTURES, load_fixture, oracle_cfg, vec_state_numpy

pytestmark = pytest.mark.gpu
REWARD_TOL = 1e-5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _vec(dev, cfg, e, **kw):
    from swarm_marl_amd import VecSwarm
    kw.setdefault("with_infos", True)
    kw.setdefault("with_global_state", True)
    return VecSwarm(e, cfg, device=dev, **kw)


# ------------------------------------------------------------------ golden fixtures
@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_golden_fixture_batched(dev, name):
    """Every recorded reference step becomes one env of a single launch (E = steps)."""
    d, raw = load_fixture(name)
    t = d["pre_pos"].shape[0]
    vec = _vec(dev, raw, t, auto_reset=False)
    vec.set_state(pos=d["pre_pos"], vel=d["pre_vel"], goal=d["pre_goal"],
                  obstacles=d["pre_obst"], active=d["pre_active"],
                  step_count=d["pre_step"].astype(np.int32))
    acts = torch.as_tensor(d["actions"]).to(dev)
    mask = torch.as_tensor(d["action_present"].astype(np.uint8)).to(dev)
    vec.step(acts, mask)
    torch.cuda.synchronize()
    obs = vec.obs.cpu().numpy()
    op = d["obs_present"]
    assert np.array_equal(obs[op], d["out_obs"][op]), "obs not bit-exact"
    rp = d["rew_present"]
    flags = vec.info_flags.cpu().numpy()
    assert np.array_equal((flags & 1).astype(bool), rp)
    assert np.array_equal((flags & 8).astype(bool), op)
    rew = vec.reward.cpu().numpy().astype(np.float64)
    if rp.any():
        assert np.abs(rew[rp] - d["rew"][rp]).max() <= REWARD_TOL
    tp = d["term_present"]
    assert np.array_equal(vec.terminated.cpu().numpy()[tp], d["term"][tp])
    assert np.array_equal(vec.truncated.cpu().numpy()[tp], d["trunc"][tp])
    env_done = vec.env_done.cpu().numpy()
    assert np.array_equal((env_done & 1).astype(bool), d["term_all"])
    assert np.array_equal((env_done & 2).astype(bool), d["trunc_all"])
    st = vec_state_numpy(vec)
    assert np.array_equal(st["pos"], d["post_pos"])
    assert np.array_equal(st["vel"], d["post_vel"])
    assert np.array_equal(st["active"], d["post_active"])
    assert np.array_equal(st["step"], d["post_step"])
    ip = d["info_present"]
    dist = vec.dist_goal.cpu().numpy()
    assert np.array_equal(dist[ip].astype(np.float64), d["info_dist"][ip])
    assert np.array_equal(((flags & 2) != 0)[ip], d["info_reached"][ip])
    assert np.array_equal(((flags & 4) != 0)[ip], d["info_collision"][ip])
    assert np.array_equal(vec.global_state.cpu().numpy(), d["global_state"])


# ------------------------------------------------------------------ oracle, multi-step
def _compare_step(vec, out, ns, tag):
    obs = vec.obs.cpu().numpy()
    if not np.array_equal(obs, out["obs"]):
        bad = np.argwhere(obs != out["obs"])
        raise AssertionError(f"{tag}: obs mismatch at {bad[:5]} (of {len(bad)})")
    err = np.abs(vec.reward.cpu().numpy().astype(np.float64) - out["reward"]).max()
    assert err <= REWARD_TOL, f"{tag}: reward err {err}"
    assert np.array_equal(vec.terminated.cpu().numpy(), out["terminated"]), tag
    assert np.array_equal(vec.truncated.cpu().numpy(), out["truncated"]), tag
    ed = vec.env_done.cpu().numpy()
    assert np.array_equal((ed & 1) != 0, out["term_all"]), tag
    assert np.array_equal((ed & 2) != 0, out["trunc_all"]), tag
    assert np.array_equal((ed & 4) != 0, out["reset"]), tag
    st = vec_state_numpy(vec)
    for k in ("pos", "vel", "goal", "obst", "active", "step", "episode", "damping"):
        assert np.array_equal(st[k], ns[k]), f"{tag}: state {k}"
    assert np.array_equal(vec.global_state.cpu().numpy(), out["global_state"]), tag
    assert np.array_equal(vec.dist_goal.cpu().numpy(), out["dist_goal"]), tag


@pytest.mark.parametrize("n,e,physics", [
    (4, 64, False), (16, 1024, False), (64, 128, False), (3, 50, False), (33, 20, False),
    (1, 40, False), (100, 6, False), (256, 3, False),
    (4, 32, True), (16, 64, True), (64, 16, True),
])
def test_oracle_multistep_autoreset(dev, n, e, physics):
    from oracle import swarm_oracle as so
    raw = dict(num_drones=n, max_steps=7)
    cfg = oracle_cfg(raw)
    vec = _vec(dev, raw, e, auto_reset=True, seed=11, env_offset=5,
               dynamics="physics" if physics else "kinematic")
    vec.reset()
    torch.cuda.synchronize()
    st = vec_state_numpy(vec)
    st_o, rout = so.reset_device(cfg, so.empty_state(cfg, e), physics=physics, seed=11,
                                 env_offset=5)
    for k in ("pos", "goal", "obst", "damping"):
        assert np.array_equal(st[k], st_o[k]), f"device reset draws differ: {k}"
    assert np.array_equal(vec.obs.cpu().numpy(), rout["obs"])
    rng = np.random.default_rng(n * 7 + e)
    for t in range(9):
        a = rng.uniform(-1.3, 1.3, (e, n, 3)).astype(np.float32)
        am = rng.uniform(size=(e, n)) > 0.15
        vec.step(torch.as_tensor(a).to(dev), torch.as_tensor(am).to(dev))
        torch.cuda.synchronize()
        st, out = so.step(cfg, st, a, am, physics=physics, auto_reset=True, seed=11,
                          env_offset=5, exact_formation=(n * e <= 20000))
        _compare_step(vec, out, st, f"N={n} E={e} phys={physics} t={t}")


@pytest.mark.parametrize("k,ms,m", [(0, 4, 8), (1, 2, 8), (2, 4, 3), (4, 4, 8), (5, 6, 8),
                                    (8, 8, 8), (12, 16, 20), (16, 0, 5), (3, 4, 0)])
def test_oracle_k_ms_variants(dev, k, ms, m):
    from oracle import swarm_oracle as so
    raw = dict(num_drones=24, neighbor_k=k, sensed_obstacles=ms, num_obstacles=m, max_steps=5)
    cfg = oracle_cfg(raw)
    e = 40
    vec = _vec(dev, raw, e, auto_reset=True, seed=3)
    vec.reset()
    torch.cuda.synchronize()
    st = vec_state_numpy(vec)
    rng = np.random.default_rng(k * 100 + ms)
    for t in range(5):
        a = rng.uniform(-1, 1, (e, 24, 3)).astype(np.float32)
        vec.step(torch.as_tensor(a).to(dev))
        torch.cuda.synchronize()
        st, out = so.step(cfg, st, a, None, auto_reset=True, seed=3)
        _compare_step(vec, out, st, f"K={k} Ms={ms} M={m} t={t}")


def test_observe_masked(dev):
    from oracle import swarm_oracle as so
    raw = dict(num_drones=16)
    cfg = oracle_cfg(raw)
    e = 33
    vec = _vec(dev, raw, e, auto_reset=False, seed=1)
    vec.reset()
    torch.cuda.synchronize()
    before = vec.obs.clone()
    st = vec_state_numpy(vec)
    mask = torch.zeros(e, dtype=torch.uint8, device=dev)
    mask[::3] = 1
    vec.reset(env_mask=mask)
    torch.cuda.synchronize()
    st2, out = so.reset_device(cfg, st, mask.cpu().numpy().astype(bool), seed=1)
    m = mask.cpu().numpy().astype(bool)
    assert np.array_equal(vec.obs.cpu().numpy()[m], out["obs"][m])
    assert torch.equal(vec.obs[~torch.as_tensor(m, device=dev)], before[~torch.as_tensor(m, device=dev)])
    st_gpu = vec_state_numpy(vec)
    for k in ("pos", "goal", "obst", "episode"):
        assert np.array_equal(st_gpu[k], st2[k])
    vec.observe()
    torch.cuda.synchronize()
    assert np.array_equal(vec.obs.cpu().numpy(), so.observe(cfg, st2["pos"], st2["vel"],
                                                            st2["goal"], st2["obst"]))


@pytest.mark.parametrize("n,k,ms,m", [(64, 3, 4, 8), (27, 3, 4, 8), (16, 8, 6, 8), (100, 5, 4, 12),
                                      (64, 16, 16, 20), (8, 4, 4, 6)])
def test_tie_heavy_lattice(dev, n, k, ms, m):
    """Drones on an integer lattice, obstacles on a symmetric sub-lattice: exact distance ties
    everywhere, which forces the exact top-K fallback (banded scan) and (distance, index)
    tie-breaking for neighbours and obstacles alike."""
    from oracle import swarm_oracle as so
    raw = dict(num_drones=n, neighbor_k=k, sensed_obstacles=ms, num_obstacles=m, max_steps=50,
               collision_radius=0.1)
    cfg = oracle_cfg(raw)
    spacings = [1.0, 0.5, 2.0, 1.5, 0.75, 1.25]
    e = len(spacings)
    side = int(np.ceil(n ** (1.0 / 3.0) - 1e-9))
    grid = np.stack(np.meshgrid(*[np.arange(side)] * 3, indexing="ij"), -1).reshape(-1, 3)[:n]
    pos = np.stack([(grid - (side - 1) / 2.0) * sp for sp in spacings]).astype(np.float32)
    ogrid = np.stack(np.meshgrid(*[np.arange(3)] * 3, indexing="ij"), -1).reshape(-1, 3)[:m]
    obst = np.stack([(ogrid - 1.0) * sp * 2.0 + 0.5 * sp for sp in spacings]).astype(np.float32)
    goal = np.tile(np.array([7.25, -6.5, 3.75], np.float32), (e, 1))
    active = np.ones((e, n), bool)
    active[-1, ::3] = False  # one env on the masked (non-fast) path
    st = dict(pos=pos, vel=np.zeros_like(pos), goal=goal, obst=obst, active=active,
              step=np.zeros(e, np.int32), episode=np.zeros(e, np.uint32),
              damping=np.zeros((e, n), np.float32))
    vec = _vec(dev, raw, e, auto_reset=False, seed=2)
    vec.set_state(pos=pos, vel=st["vel"], goal=goal, obstacles=obst, active=active,
                  step_count=st["step"])
    for t in range(2):
        a = np.zeros((e, n, 3), np.float32)
        vec.step(torch.as_tensor(a).to(dev))
        torch.cuda.synchronize()
        st, out = so.step(cfg, st, a, None, auto_reset=False, seed=2, exact_formation=True)
        _compare_step(vec, out, st, f"lattice N={n} K={k} Ms={ms} M={m} t={t}")


@pytest.mark.parametrize("n,e,radii", [(128, 6, 0.0), (256, 3, 0.0), (256, 4, 0.5), (512, 2, 0.0), (128, 5, 0.5)])
def test_block_rotation_passes_vs_oracle(dev, n, e, radii):
    """Block teams with N a power of two run the rotation passes over the pair-entry ring: the
    step's formation/minimum pass, then (envs that do not reset) a keys pass, or the reset's
    keys pass.  radii 0 (no collisions, no goals: no resets until max_steps) exercises the
    continuing path; default radii the reset path."""
    from oracle import swarm_oracle as so
    raw = dict(num_drones=n, max_steps=6, collision_radius=radii, goal_radius=radii,
               obstacle_radius=radii if radii else 0.0)
    cfg = oracle_cfg(raw)
    vec = _vec(dev, raw, e, auto_reset=True, seed=17, env_offset=3)
    vec.reset()
    torch.cuda.synchronize()
    st = vec_state_numpy(vec)
    rng = np.random.default_rng(n + e)
    resets = 0
    for t in range(8):
        a = rng.uniform(-1.2, 1.2, (e, n, 3)).astype(np.float32)
        vec.step(torch.as_tensor(a).to(dev))
        torch.cuda.synchronize()
        st, out = so.step(cfg, st, a, None, auto_reset=True, seed=17, env_offset=3, exact_formation=(n * e <= 20000))
        _compare_step(vec, out, st, f"N={n} E={e} radii={radii} t={t}")
        resets += int((vec.env_done.cpu().numpy() & 4).astype(bool).sum())
    if radii == 0.0:
        assert resets == e  # only the max_steps truncation at t = 5
