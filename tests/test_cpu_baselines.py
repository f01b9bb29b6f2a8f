"""CPU: the bench's CPU-baseline variants are faithful restatements, pinned to the reference.

* oracle/swarm_loop.py (BASELINE.md §5 variant (a), per-agent loops like the reference) must
  reproduce every recorded reference step bit-exactly: observations, float64 rewards, flags,
  "__all__" and the post-step state; and the seeded reset draws.
* bench.py's CPU-baseline helpers run a bounded sample and report the fields the bench line needs.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import ROLLOUT_FIXTURES, load_fixture


def _loop_env(raw, d, row):
    from oracle.swarm_loop import LoopSwarm
    cfg = {k: v for k, v in raw.items() if k not in ("num_drones", "seed")}
    env = LoopSwarm(int(raw.get("num_drones", 3)), **cfg)
    env.pos = d["pre_pos"][row].copy()
    env.vel = d["pre_vel"][row].copy()
    env.goal = d["pre_goal"][row].copy()
    env.obst = d["pre_obst"][row].copy()
    env.t = int(d["pre_step"][row])
    env.live = [i for i in range(env.n) if d["pre_active"][row, i]]
    return env


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_loop_restatement_matches_reference_fixture(name):
    d, raw = load_fixture(name)
    for row in range(d["pre_pos"].shape[0]):
        env = _loop_env(raw, d, row)
        acts = {env.ids[i]: d["actions"][row, i] for i in range(env.n) if d["action_present"][row, i]}
        obs, rew, term, trunc, info = env.step(acts)
        for i, aid in enumerate(env.ids):
            assert (aid in obs) == bool(d["obs_present"][row, i])
            if aid in obs:
                assert np.array_equal(obs[aid], d["out_obs"][row, i]), (name, row, aid)
                assert info[aid]["distance_to_goal"] == d["info_dist"][row, i]
                assert np.array_equal(info[aid]["global_state"], d["global_state"][row])
            assert (aid in rew) == bool(d["rew_present"][row, i])
            if aid in rew:
                assert rew[aid] == d["rew"][row, i], (name, row, aid)  # bit-exact float64
                assert term[aid] == bool(d["term"][row, i])
                assert trunc[aid] == bool(d["trunc"][row, i])
        assert term["__all__"] == bool(d["term_all"][row])
        assert trunc["__all__"] == bool(d["trunc_all"][row])
        assert np.array_equal(env.pos, d["post_pos"][row])
        assert np.array_equal(env.vel, d["post_vel"][row])
        assert env.t == int(d["post_step"][row])
        assert [bool(i in env.live) for i in range(env.n)] == d["post_active"][row].tolist()


@pytest.mark.parametrize("name", ["reset_n4.npz", "reset_n64.npz"])
def test_loop_restatement_seeded_reset(name):
    from oracle.swarm_loop import LoopSwarm
    d, raw = load_fixture(name)
    cfg = {k: v for k, v in raw.items() if k not in ("num_drones", "seed")}
    env = LoopSwarm(int(raw["num_drones"]), **cfg)
    for k, s in enumerate(d["seeds"]):
        obs, info = env.reset(seed=int(s))
        assert np.array_equal(env.pos, d["seeded_pos"][k])
        assert np.array_equal(env.goal, d["seeded_goal"][k])
        assert np.array_equal(env.obst, d["seeded_obst"][k])
        got = np.stack([obs[a] for a in env.ids])
        assert np.array_equal(got, d["seeded_obs"][k])
        assert np.array_equal(info[env.ids[0]]["global_state"], d["seeded_global_state"][k])


def test_loop_run_for_counts_agent_steps():
    from oracle.swarm_loop import run_for
    count, el = run_for(2, 4, 0.05)
    assert count > 0 and el >= 0.05


def test_bench_cpu_variants_small():
    import bench
    rec = bench.cpu_python_variants(n=4, e=4, seconds=0.2, procs=2)
    assert [r["kind"] for r in rec] == ["port", "port"]
    for r in rec:
        assert r["value"] > 0 and r["cores"] == 2 and r["unit"] == "agent-steps/s"
        assert "restatement" in r["sample"]
