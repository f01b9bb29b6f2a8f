"""CPU: host-side logic of the drop-in package (no GPU compute).

- DroneEnvConfig mirrors the reference's config (src/swarm_marl/envs/common.py:7-32).
- Seeded host reset draws reproduce the reference's NumPy stream (drone_swarm_env.py:62-80),
  pinned by tests/golden/reset_n4.npz / reset_n64.npz (seeded and continued streams).
- build_step_dicts turns the kernel's dense outputs into the reference's RLlib dicts
  (drone_swarm_env.py:129-174), pinned by the rollout fixtures' presence masks and values.
"""
from __future__ import annotations

import json

import numpy as np
import pytest

from tests.helpers import GOLDEN, ROLLOUT_FIXTURES, load_fixture


def test_config_defaults_and_from_dict():
    from swarm_marl_amd.envs.common import DroneEnvConfig
    c = DroneEnvConfig()
    assert (c.world_size, c.dt, c.max_steps, c.max_speed, c.max_accel) == (20.0, 0.1, 400, 4.0, 2.0)
    assert (c.collision_radius, c.goal_radius, c.num_obstacles, c.sensed_obstacles) == (0.5, 0.8, 8, 4)
    assert (c.neighbor_k, c.obstacle_radius, c.desired_spacing) == (3, 0.8, 2.5)
    assert (c.reward_progress_scale, c.reward_goal, c.reward_collision) == (2.0, 25.0, -25.0)
    assert c.reward_formation_scale == 0.15 and c.seed is None
    c2 = DroneEnvConfig.from_dict({"max_steps": 7, "num_drones": 9, "bogus": 1})
    assert c2.max_steps == 7 and not hasattr(c2, "bogus")
    assert DroneEnvConfig.from_dict(None) == DroneEnvConfig()
    assert c.obs_dim() == 9 + 4 * 3 + 4 * 4 == 37
    assert c.obs_dim(with_neighbors=False) == 25


@pytest.mark.parametrize("fixture,n", [("reset_n4.npz", 4), ("reset_n64.npz", 64)])
def test_seeded_host_reset_matches_reference(fixture, n):
    from oracle import swarm_oracle as so
    from swarm_marl_amd.envs.host_reset import swarm_reset_draws
    d = np.load(GOLDEN / fixture)
    cfg = json.loads(str(d["config"]))
    for i, s in enumerate(d["seeds"]):
        pos, goal, obst = swarm_reset_draws(np.random.default_rng(int(s)), n, 8, 20.0)
        assert np.array_equal(pos, d["seeded_pos"][i])
        assert np.array_equal(goal, d["seeded_goal"][i])
        assert np.array_equal(obst, d["seeded_obst"][i])
    # reset() without a seed continues the stream created from cfg.seed
    rng = np.random.default_rng(cfg.get("seed"))
    for i in range(d["cont_pos"].shape[0]):
        pos, goal, obst = swarm_reset_draws(rng, n, 8, 20.0)
        assert np.array_equal(pos, d["cont_pos"][i])
        assert np.array_equal(goal, d["cont_goal"][i])
        assert np.array_equal(obst, d["cont_obst"][i])
    # reset observations and distances (observe pass of the reset)
    ocfg = so.make_cfg(**cfg)
    obs = so.observe(ocfg, d["seeded_pos"], d["seeded_vel"], d["seeded_goal"], d["seeded_obst"])
    assert np.array_equal(obs, d["seeded_obs"])
    gs = so.global_state(d["seeded_pos"], d["seeded_vel"], d["seeded_goal"])
    assert np.array_equal(gs, d["seeded_global_state"])


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES[:8])
def test_build_step_dicts_matches_reference_dicts(name):
    """Dense kernel outputs (taken from the fixture) -> dict presence/value semantics."""
    from swarm_marl_amd import _native as nat
    from swarm_marl_amd.envs.drone_swarm_env import build_step_dicts
    d, _ = load_fixture(name)
    t, n = d["rew_present"].shape
    ids = [f"drone_{i}" for i in range(n)]
    for s in range(t):
        flags = (d["rew_present"][s] * nat.AGENT_STEPPED
                 | (d["info_reached"][s] & d["info_present"][s]) * nat.AGENT_REACHED
                 | (d["info_collision"][s] & d["info_present"][s]) * nat.AGENT_COLLISION
                 | d["obs_present"][s] * nat.AGENT_HAS_OBS).astype(np.uint8)
        env_done = int(d["term_all"][s]) * nat.ENV_TERMINATED | int(d["trunc_all"][s]) * nat.ENV_TRUNCATED
        obs_d, rew_d, term_d, trunc_d, info_d = build_step_dicts(
            ids, d["out_obs"][s], d["rew"][s], d["term"][s], d["trunc"][s], flags,
            d["info_dist"][s], d["global_state"][s], env_done)
        assert set(rew_d) == {ids[i] for i in np.nonzero(d["rew_present"][s])[0]}
        assert set(obs_d) == {ids[i] for i in np.nonzero(d["obs_present"][s])[0]}
        assert set(info_d) == {ids[i] for i in np.nonzero(d["info_present"][s])[0]}
        assert term_d["__all__"] == bool(d["term_all"][s])
        assert trunc_d["__all__"] == bool(d["trunc_all"][s])
        for i in np.nonzero(d["rew_present"][s])[0]:
            assert rew_d[ids[i]] == d["rew"][s, i]
            assert term_d[ids[i]] == bool(d["term"][s, i])
            assert trunc_d[ids[i]] == bool(d["trunc"][s, i])
        for i in np.nonzero(d["info_present"][s])[0]:
            inf = info_d[ids[i]]
            assert inf["distance_to_goal"] == d["info_dist"][s, i]
            assert inf["reached_goal"] == bool(d["info_reached"][s, i])
            assert inf["collision"] == bool(d["info_collision"][s, i])
            assert np.array_equal(inf["global_state"], d["global_state"][s])
            assert np.array_equal(obs_d[ids[i]], d["out_obs"][s, i])


def test_shard_bounds_partition():
    from swarm_marl_amd.distributed import shard_bounds
    for total in (0, 1, 7, 8192, 65537):
        for ws in (1, 2, 3, 8):
            spans = [shard_bounds(total, ws, r) for r in range(ws)]
            assert spans[0][0] == 0
            for (o0, c0), (o1, _) in zip(spans, spans[1:]):
                assert o0 + c0 == o1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)
