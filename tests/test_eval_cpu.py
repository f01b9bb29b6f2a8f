"""CPU: the eval-metric oracle (oracle/eval_oracle.py) against the reference's own metric code.

tests/golden/eval_*.npz were produced by the reference's evaluate_protocol.py metric functions
(:103-116, :237-331, :334-350) driving the reference DroneSwarmEnv (make_eval_golden.py).  Each
recorded episode is replayed here through the per-agent restatement of the env
(oracle/swarm_loop.py, itself pinned bit-exactly to the reference step fixtures) and the
restated metrics must reproduce every EpisodeSummary field and the aggregate.
"""
from __future__ import annotations

import json
import math

import numpy as np
import pytest

from tests.conftest import GOLDEN

EVAL_FIXTURES = sorted(p.name for p in GOLDEN.glob("eval_*.npz"))


def replay_episode(d, cfg, k):
    """(reset obs, [(obs, rew, term, trunc, infos)...]) of recorded episode k through LoopSwarm."""
    from oracle.swarm_loop import LoopSwarm
    raw = dict(cfg)
    n = int(raw.pop("num_drones", 3))
    raw.pop("seed", None)
    env = LoopSwarm(n, **raw)
    env.pos = d["reset_pos"][k].copy()
    env.vel = np.zeros((n, 3), np.float32)
    env.goal = d["reset_goal"][k].copy()
    env.obst = d["reset_obst"][k].copy()
    env.live, env.t = list(range(n)), 0
    reset_obs = {env.ids[i]: env.observe(i) for i in range(n)}
    outs = []
    for t in range(int(d["lengths"][k])):
        acts = {env.ids[i]: d["actions"][k, t, i] for i in range(n) if d["present"][k, t, i]}
        outs.append(env.step(acts))
    return reset_obs, outs


@pytest.mark.parametrize("name", EVAL_FIXTURES)
def test_eval_oracle_matches_reference(name):
    from oracle import eval_oracle as ev
    d = np.load(GOLDEN / name)
    cfg = json.loads(str(d["config"]))
    spacing = float(cfg.get("desired_spacing", 2.5))
    sums = []
    for k in range(len(d["lengths"])):
        reset_obs, outs = replay_episode(d, cfg, k)
        m = ev.EpisodeMetrics(reset_obs, spacing)
        for t, o in enumerate(outs):
            done = m.update(*o)
            assert done == (t == len(outs) - 1), (name, k, t)
        s = m.summary()
        exp = d["summaries"][k]
        for f, (a, b) in enumerate(zip(s, exp)):
            assert (math.isnan(a) and math.isnan(b)) or a == pytest.approx(b, rel=1e-12, abs=1e-12), (name, k, f)
        sums.append(s)
    agg = ev.aggregate(sums)
    ref = json.loads(str(d["aggregate"]))
    for key, v in ref.items():
        assert (isinstance(v, float) and math.isnan(v) and math.isnan(agg[key])) or agg[key] == pytest.approx(v, rel=1e-12), key


EVAL1_FIXTURES = sorted(p.name for p in GOLDEN.glob("eval1_*.npz"))


def single_env(d, cfg, k):
    """LoopSwarm with one drone and no neighbours at recorded episode k's reset state."""
    from oracle.swarm_loop import LoopSwarm
    raw = dict(cfg)
    raw.pop("seed", None)
    env = LoopSwarm(1, neighbor_k=0, **raw)
    env.pos = d["reset_pos"][k].reshape(1, 3).copy()
    env.vel = np.zeros((1, 3), np.float32)
    env.goal = d["reset_goal"][k].copy()
    env.obst = d["reset_obst"][k].copy()
    env.live, env.t = [0], 0
    return env


@pytest.mark.parametrize("name", EVAL1_FIXTURES)
def test_single_agent_eval_oracle_matches_reference(name):
    """evaluate_protocol.py:193-234 over the reference SingleDroneEnv (eval1_*.npz): goal
    reached, collision (SR = CFR = 0) and time-limit (NaN TTG) episodes."""
    from oracle import eval_oracle as ev
    d = np.load(GOLDEN / name)
    cfg = json.loads(str(d["config"]))
    sums = []
    for k in range(len(d["lengths"])):
        env = single_env(d, cfg, k)
        m = ev.SingleEpisodeMetrics(env.observe(0))
        n = int(d["lengths"][k])
        for t in range(n):
            done = m.update(*ev.single_drone_step(env, d["actions"][k, t]))
            assert done == (t == n - 1), (name, k, t)
        s = m.summary()
        for f, (a, b) in enumerate(zip(s, d["summaries"][k])):
            assert (math.isnan(a) and math.isnan(b)) or a == pytest.approx(b, rel=1e-12, abs=1e-12), (name, k, f)
        sums.append(s)
    agg = ev.aggregate(sums)
    for key, v in json.loads(str(d["aggregate"])).items():
        assert (isinstance(v, float) and math.isnan(v) and math.isnan(agg[key])) or agg[key] == pytest.approx(v, rel=1e-12), key


def test_single_agent_fixtures_cover_failure_branches():
    """The eval1 fixtures hold successes, collisions and time-limit episodes (the branches the
    swarm protocol's fixtures cannot reach)."""
    sm = np.concatenate([np.load(GOLDEN / n)["summaries"] for n in EVAL1_FIXTURES])
    assert (sm[:, 0] == 1).any() and (sm[:, 0] == 0).any()
    assert (sm[:, 1] == 0).any() and np.isnan(sm[:, 2]).any()


# ---------------------------------------------------------------- curriculum / aggregation host logic
STAGES = {"promotion_window_episodes": 4, "stages": [
    {"stage_id": 1, "stage_name": "a", "env_config": {"num_drones": 3, "num_obstacles": 0, "max_steps": 30},
     "train_iterations": 2, "promotion_criteria": {"min_success_rate": 0.5, "min_collision_free_rate": 0.5,
                                                   "max_mean_time_to_goal": 40}},
    {"stage_id": 2, "stage_name": "b", "env_config": {"num_drones": 5, "num_obstacles": 4, "max_steps": 30,
                                                      "world_size": 24.0}, "train_iterations": 1}]}


def test_curriculum_yaml_roundtrip(tmp_path):
    import yaml
    from swarm_marl_amd.curriculum import load_curriculum, stage_env_config
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(STAGES))
    cfg = load_curriculum(p)
    assert stage_env_config(cfg, 1, base_seed=7) == {"num_drones": 5, "num_obstacles": 4, "max_steps": 30,
                                                     "world_size": 24.0, "seed": 8}
    bad = tmp_path / "bad.yaml"
    bad.write_text("stages: []\n")
    with pytest.raises(ValueError):
        load_curriculum(bad)


def test_reference_curriculum_parses():
    from pathlib import Path
    from swarm_marl_amd.curriculum import load_curriculum
    ref = Path("/root/reference/configs/curriculum_v1.yaml")
    if not ref.exists():
        pytest.skip("reference configs not present (GPU box)")
    cfg = load_curriculum(ref)
    assert [s["env_config"]["num_drones"] for s in cfg["stages"]] == [3, 3, 5, 8]


def test_criteria_and_aggregate():
    from swarm_marl_amd.curriculum import criteria_met
    from swarm_marl_amd.eval_metrics import aggregate_records
    rec = np.array([[0, 1, 1, 10, 2.0, 1.0, 5.0, 10], [1, 0, 1, np.nan, 3.0, 0.5, -5.0, 30]], np.float64)
    m = aggregate_records(rec)
    from oracle import eval_oracle as ev
    ref = ev.aggregate([tuple(r[1:7]) for r in rec])
    for k, v in ref.items():
        assert (math.isnan(v) and math.isnan(m[k])) or m[k] == pytest.approx(v), k
    crit = STAGES["stages"][0]["promotion_criteria"]
    assert criteria_met(m, crit)
    assert not criteria_met(dict(m, success_rate=0.4), crit)
    assert not criteria_met(dict(m, mean_time_to_goal=math.nan), crit)
    assert criteria_met(m, None)
