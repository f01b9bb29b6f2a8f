"""GPU: per-env parameters (swarm_env_cfg_t; SURVEY.md §8f row 4 — curriculum stages and domain
randomisation as per-env tensors) through the C-ABI.

* uniform records change nothing: a batch given records that hold the batch config equals the
  batch without records bit for bit (wave teams, the N = 64 path — generic kernel vs step64 —,
  block teams, physics), over steps with in-kernel resets;
* per-env values (world size, dt, speed / accel limits, obstacle radius, episode length, active
  obstacle count incl. fewer than Ms and zero) match the oracle stepping each env with its own
  config (oracle/env_cfg_oracle.py): obs bit-exact, rewards within 1e-5, flags and state exact;
* next-episode records: every reset (auto or explicit) switches the env to them, as the oracle.
Reference: src/swarm_marl/envs/drone_swarm_env.py:28-174 (one config per env instance),
configs/curriculum_v1.yaml:9-60, configs/domain_randomization_v1.yaml:9-57.
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


def _actions(dev, t, e, n, scale=1.0):
    g = torch.Generator(device=dev).manual_seed(9100 + t)
    return (torch.rand((e, n, 3), device=dev, generator=g) * 2 - 1) * scale


def _snap(vec):
    return [t.clone() for t in (vec.obs, vec.reward, vec.terminated, vec.truncated, vec.env_done,
                                vec.pos, vec.vel, vec.goal, vec.obstacles, vec.active,
                                vec.step_count, vec.episode, vec.damping)]


@pytest.mark.parametrize("n,e,dyn,groups", [(16, 64, "kinematic", 1), (64, 24, "kinematic", 2),
                                            (256, 6, "kinematic", 1), (8, 32, "physics", 1)])
def test_uniform_records_equal_no_records(dev, n, e, dyn, groups):
    from swarm_marl_amd import VecSwarm
    cfg = {"num_drones": n, "max_steps": 7}
    # N = 16 / 64 / 256 without records run swarm_step16q / swarm_step64_once / swarm_step256w, whose
    # kinematic rewards equal the generic kernel's within 1e-5 only (formation partial sums in
    # another order; tests/test_gpu_step16.py, test_gpu_step64.py, test_gpu_step256.py): compare
    # the records path with the generic kernel there
    kp = "generic" if n in (16, 64, 256) and dyn == "kinematic" else "auto"
    a_vec = VecSwarm(e, cfg, device=dev, auto_reset=True, seed=11, dynamics=dyn, groups=groups, kernel_path=kp)
    b_vec = VecSwarm(e, cfg, device=dev, auto_reset=True, seed=11, dynamics=dyn, groups=groups)
    b_vec.set_env_config()  # records holding the batch config
    assert b_vec.kernel_name().startswith("swarm_kernel<")
    if kp == "generic":  # the records path's name is the generic kernel's, lane mode included
        assert b_vec.kernel_name() == a_vec.kernel_name()
    a_vec.reset()
    b_vec.reset()
    resets = 0
    for t in range(16):
        a = _actions(dev, t, e, n)
        a_vec.step(a)
        b_vec.step(a)
        for k, (x, y) in enumerate(zip(_snap(a_vec), _snap(b_vec))):
            assert torch.equal(x, y), f"t={t} field {k}"
        resets += int(((a_vec.env_done & 4) != 0).sum())
    assert resets >= e, "the run must cross episode boundaries"


def _overrides(e, m, rng, physics=False):
    ov = dict(world_size=rng.uniform(12.0, 30.0, e), max_speed=rng.uniform(2.0, 6.0, e),
              max_accel=rng.uniform(1.0, 3.5, e), obstacle_radius=rng.uniform(0.4, 1.4, e),
              max_steps=rng.integers(4, 12, e).astype(np.int32),
              num_obstacles=np.resize(np.array([0, 1, 3, m, m - 1, 2], np.int32), e))
    if not physics:
        ov["dt"] = rng.uniform(0.05, 0.2, e)
    return ov


def _compare(vec, ns, out, t, what):
    obs = vec.obs.cpu().numpy()
    assert np.array_equal(obs, out["obs"]), f"{what} t={t}: obs differ in {np.argwhere(obs != out['obs'])[:4]}"
    err = np.abs(vec.reward.cpu().numpy().astype(np.float64) - out["reward"]).max()
    assert err < REWARD_TOL, f"{what} t={t}: reward error {err}"
    assert np.array_equal(vec.terminated.cpu().numpy(), out["terminated"]), f"{what} t={t}"
    assert np.array_equal(vec.truncated.cpu().numpy(), out["truncated"]), f"{what} t={t}"
    bits = out["term_all"].astype(np.uint8) | (out["trunc_all"].astype(np.uint8) << 1) | \
        (out["reset"].astype(np.uint8) << 2)
    assert np.array_equal(vec.env_done.cpu().numpy(), bits), f"{what} t={t}"
    st = vec_state_numpy(vec)
    for k in ("pos", "vel", "goal", "obst", "active", "step", "episode"):
        assert np.array_equal(st[k], ns[k]), f"{what} t={t}: state {k}"


@pytest.mark.parametrize("n,e,m,dyn,steps", [(8, 12, 8, "kinematic", 18), (3, 20, 6, "kinematic", 14),
                                              (64, 4, 8, "kinematic", 6), (128, 3, 6, "kinematic", 5),
                                              (4, 8, 5, "physics", 12)])
def test_per_env_params_vs_oracle(dev, n, e, m, dyn, steps):
    from oracle import env_cfg_oracle as eco
    from swarm_marl_amd import VecSwarm
    physics = dyn == "physics"
    raw = {"num_drones": n, "num_obstacles": m}
    base = oracle_cfg(raw)
    rng = np.random.default_rng(n * 100 + e)
    ov = _overrides(e, m, rng, physics)
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=23, dynamics=dyn)
    vec.set_env_config(**ov)
    st0 = vec_state_numpy(vec)
    vec.reset()
    torch.cuda.synchronize()
    ns, ro = eco.reset(base, ov, st0, seed=23, physics=physics)
    assert np.array_equal(vec.obs.cpu().numpy(), ro["obs"]), "reset obs"
    st = vec_state_numpy(vec)
    for k in ("pos", "goal", "obst"):
        assert np.array_equal(st[k], ns[k]), f"reset state {k}"
    cfgv = vec.env_config()
    assert np.array_equal(cfgv["num_obstacles"].cpu().numpy(), np.clip(ov["num_obstacles"], 0, m))
    assert np.array_equal(cfgv["world_size"].cpu().numpy(), ov["world_size"])
    resets = 0
    for t in range(steps):
        a = _actions(dev, t, e, n, scale=2.0)
        st = vec_state_numpy(vec)
        vec.step(a)
        torch.cuda.synchronize()
        ns, out, _ = eco.step(base, ov, st, a.cpu().numpy(), seed=23, physics=physics)
        _compare(vec, ns, out, t, f"N={n} {dyn}")
        resets += int(out["reset"].sum())
    assert resets > 0


def test_next_episode_params_vs_oracle(dev):
    from oracle import env_cfg_oracle as eco
    from swarm_marl_amd import VecSwarm
    n, e, m = 8, 16, 8
    raw = {"num_drones": n, "num_obstacles": m}
    base = oracle_cfg(raw)
    rng = np.random.default_rng(5)
    cur = _overrides(e, m, rng)
    nxt = _overrides(e, m, rng)
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=31, with_infos=True)
    vec.set_env_config(**cur)
    ns, _ = eco.reset(base, cur, vec_state_numpy(vec), seed=31)
    vec.reset()
    torch.cuda.synchronize()
    st0 = vec_state_numpy(vec)
    assert np.array_equal(st0["pos"], ns["pos"]) and np.array_equal(st0["obst"], ns["obst"])
    vec.set_env_config(next_episode=True, **nxt)
    # explicit reset of half the envs: they switch to the next-episode values at once
    mask = torch.zeros(e, dtype=torch.bool, device=dev)
    mask[::2] = True
    vec.reset(mask)
    torch.cuda.synchronize()
    ns, _ = eco.reset(base, cur, st0, nxt=nxt, env_mask=mask.cpu().numpy(), seed=31)
    st = vec_state_numpy(vec)
    for k in ("pos", "vel", "goal", "obst", "active", "step", "episode"):
        assert np.array_equal(st[k], ns[k]), f"explicit reset state {k}"
    ws = vec.env_config()["world_size"].cpu().numpy()
    assert np.array_equal(ws[::2], nxt["world_size"][::2]) and np.array_equal(ws[1::2], cur["world_size"][1::2])
    live = {k: np.where(np.arange(e) % 2 == 0, nxt[k], cur[k]).astype(np.asarray(cur[k]).dtype) for k in cur}
    resets = 0
    for t in range(14):
        a = _actions(dev, t, e, n, scale=2.0)
        st = vec_state_numpy(vec)
        vec.step(a)
        torch.cuda.synchronize()
        ns, out, live = eco.step(base, live, st, a.cpu().numpy(), nxt=nxt, seed=31)
        _compare(vec, ns, out, t, "next-episode")
        got = vec.env_config()
        assert np.array_equal(got["world_size"].cpu().numpy(), live["world_size"]), f"t={t} world_size"
        assert np.array_equal(got["max_steps"].cpu().numpy(), live["max_steps"]), f"t={t} max_steps"
        resets += int(out["reset"].sum())
    assert resets >= e // 2


def test_curriculum_mixed_stages_vs_oracle(dev):
    """Stages 1 and 2 of curriculum_v1 (both N = 3) in ONE batch: per-env num_obstacles,
    max_steps, world_size; each env equals the oracle with its stage's env_config."""
    from oracle import env_cfg_oracle as eco
    from swarm_marl_amd.curriculum import mixed_stage_batch
    cfg = {"stages": [
        {"env_config": {"num_drones": 3, "num_obstacles": 0, "max_steps": 9, "world_size": 20.0}},
        {"env_config": {"num_drones": 3, "num_obstacles": 4, "max_steps": 6, "world_size": 24.0}}]}
    stage_of_env = [0, 1] * 8
    vec, over = mixed_stage_batch(cfg, stage_of_env, device=dev, seed=41)
    base = oracle_cfg({"num_drones": 3, "num_obstacles": 4})
    vec.reset()
    torch.cuda.synchronize()
    e = len(stage_of_env)
    for t in range(12):
        a = _actions(dev, t, e, 3, scale=2.0)
        st = vec_state_numpy(vec)
        vec.step(a)
        torch.cuda.synchronize()
        ns, out, _ = eco.step(base, over, st, a.cpu().numpy(), seed=41)
        _compare(vec, ns, out, t, "curriculum mix")


def test_domain_randomizer_draws_per_episode(dev):
    """Each reset env starts the parameters drawn for it ahead of time; after the step it gets
    fresh next-episode draws, the others keep theirs (all on the device)."""
    import yaml
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.domain_randomization import DomainRandomizer
    from tests.test_env_cfg_cpu import DR_YAML
    e, n = 64, 8
    vec = VecSwarm(e, {"num_drones": n, "max_steps": 4}, device=dev, auto_reset=True, seed=2)
    dr = DomainRandomizer(vec, yaml.safe_load(DR_YAML), seed=1, force=True)
    assert "dynamics.mass_scale" in dr.unsupported
    dr.begin()  # resets, then queues a fresh draw for every env's next episode
    torch.cuda.synchronize()
    cur = vec.env_config()
    ws = cur["world_size"].cpu().numpy()
    assert ws.min() >= 19.0 and ws.max() <= 21.0 and len(np.unique(ws)) == e
    assert np.allclose(cur["half_w"].cpu().numpy(), (ws / 2.0).astype(np.float32))
    nxt = vec.env_config(True)
    for k in ("world_size", "max_speed", "max_accel", "dt"):  # episodes 1 and 2 differ per env
        assert bool((cur[k] != nxt[k]).all()), k
    # an explicit reset consumes the queued draw; after_reset refills it
    queued = {k: v.clone() for k, v in nxt.items()}
    vec.reset()
    dr.after_reset()
    torch.cuda.synchronize()
    cur, nxt = vec.env_config(), vec.env_config(True)
    for k in ("world_size", "max_speed", "max_accel", "dt"):
        assert torch.equal(cur[k], queued[k]), k
        assert bool((cur[k] != nxt[k]).all()), k
    switched = 0
    for t in range(6):
        prev_cur = {k: v.clone() for k, v in vec.env_config().items()}
        prev_next = {k: v.clone() for k, v in vec.env_config(True).items()}
        vec.step(_actions(dev, t, e, n, scale=2.0))
        dr.after_step()
        torch.cuda.synchronize()
        reset = ((vec.env_done & 4) != 0)
        now_cur, now_next = vec.env_config(), vec.env_config(True)
        for k in ("world_size", "max_speed", "max_accel", "dt"):
            assert torch.equal(now_cur[k][reset], prev_next[k][reset]), (t, k)
            assert torch.equal(now_cur[k][~reset], prev_cur[k][~reset]), (t, k)
            assert torch.equal(now_next[k][~reset], prev_next[k][~reset]), (t, k)
            assert bool((now_next[k][reset] != prev_next[k][reset]).all()), (t, k)
        switched += int(reset.sum())
    assert switched >= e
