"""GPU: on-device eval metrics (swarm_eval_update / EvalTracker) against the reference's metric
code and its restatement.

* Every episode of tests/golden/eval_*.npz (the reference's evaluate_protocol.py metric functions
  on the reference DroneSwarmEnv, make_eval_golden.py) is replayed as one env of a VecSwarm from
  its recorded reset state and actions: success, collision-free and time-to-goal exact,
  formation error and path efficiency to 1e-9 relative, episode reward within the per-step
  reward contract (1e-5 x steps), and the `_aggregate` dict.
* With in-kernel auto-reset (episodes rolling over inside the launch), every record equals the
  oracle's (oracle/eval_oracle.py) summary of the same env's episode, fed the dict outputs.
"""
from __future__ import annotations

import json
import math

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu
EVAL_FIXTURES = sorted(p.name for p in GOLDEN.glob("eval_*.npz"))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _cmp_summary(got, exp, steps, tag):
    assert got[1] == exp[0] and got[2] == exp[1], tag
    assert (math.isnan(got[3]) and math.isnan(exp[2])) or got[3] == exp[2], tag
    assert got[4] == pytest.approx(exp[3], rel=1e-9, abs=1e-12), tag
    assert got[5] == pytest.approx(exp[4], rel=1e-9, abs=1e-12), tag
    assert abs(got[6] - exp[5]) <= 1e-5 * steps + 1e-9, tag


@pytest.mark.parametrize("name", EVAL_FIXTURES)
def test_eval_replays_reference_episodes(dev, name):
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import EvalTracker
    d = np.load(GOLDEN / name)
    cfg = json.loads(str(d["config"]))
    n = int(cfg["num_drones"])
    lens = d["lengths"]
    e = len(lens)
    vec = VecSwarm(e, cfg, device=dev, auto_reset=False, with_infos=True)
    vec.set_state(pos=d["reset_pos"], vel=np.zeros((e, n, 3), np.float32), goal=d["reset_goal"],
                  obstacles=d["reset_obst"], active=np.ones((e, n), bool), step_count=np.zeros(e, np.int32))
    vec.observe()
    ev = EvalTracker(vec, capacity=64)
    ev.begin()
    acts = torch.as_tensor(d["actions"], device=dev)
    for t in range(int(lens.max()) + 2):  # two steps past the last end: finished envs stay closed
        vec.step(acts[:, t].contiguous() if t < acts.shape[1] else torch.zeros((e, n, 3), device=dev))
        ev.update()
    rec = ev.records()
    assert len(rec) == e
    rec = rec[np.argsort(rec[:, 0], kind="stable")]
    for k in range(e):
        assert int(rec[k, 7]) == int(lens[k])
        _cmp_summary(rec[k], d["summaries"][k], int(lens[k]), (name, k))
    agg, ref = ev.aggregate(), json.loads(str(d["aggregate"]))
    for key in ("success_rate", "collision_free_rate", "mean_time_to_goal"):
        assert agg[key] == ref[key], key
    for key in ("formation_error", "path_efficiency"):
        assert agg[key] == pytest.approx(ref[key], rel=1e-9), key
    assert agg["episode_reward_mean"] == pytest.approx(ref["episode_reward_mean"], abs=1e-3)


@pytest.mark.parametrize("n", [8, 16, 33, 40])
def test_eval_auto_reset_matches_oracle(dev, n):
    """The unfused update kernel (not N = 64) against the oracle's episode metrics with
    auto-reset: N = 8 / 16 take the small-swarm formation path (several lanes per drone), N = 33 /
    40 the general symmetric-rotation one (odd N, and even N with its opposite pairs)."""
    from oracle import eval_oracle as ev_o
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd import _native as nat
    from swarm_marl_amd.envs.drone_swarm_env import build_step_dicts
    from swarm_marl_amd.eval_metrics import EvalTracker
    e, steps = (96, 60) if n <= 16 else (32, 40)
    vec = VecSwarm(e, {"num_drones": n, "max_steps": 25}, device=dev, auto_reset=True, seed=5, with_infos=True,
                   with_global_state=True, groups=2)
    vec.reset()
    ev = EvalTracker(vec, capacity=4096)
    ev.begin()
    ids = [f"drone_{i}" for i in range(n)]

    def reset_obs(o, i):
        return {a: o[i, k].copy() for k, a in enumerate(ids)}

    obs0 = vec.obs.cpu().numpy()
    trackers = [ev_o.EpisodeMetrics(reset_obs(obs0, i), 2.5) for i in range(e)]
    expected = []
    g = torch.Generator(device=dev).manual_seed(9)
    for t in range(steps):
        vec.step(torch.rand((e, n, 3), device=dev, generator=g) * 2 - 1)
        ev.update()
        o, r = vec.obs.cpu().numpy(), vec.reward.cpu().numpy()
        te, tr = vec.terminated.cpu().numpy(), vec.truncated.cpu().numpy()
        fl, dg = vec.info_flags.cpu().numpy(), vec.dist_goal.cpu().numpy()
        gs, done = vec.global_state.cpu().numpy(), vec.env_done.cpu().numpy()
        for i in range(e):
            outs = build_step_dicts(ids, o[i], r[i], te[i], tr[i], fl[i], dg[i], gs[i], int(done[i]))
            if trackers[i].update(*outs):
                expected.append((i, trackers[i].summary(), trackers[i].steps))
                assert done[i] & nat.ENV_RESET
                trackers[i] = ev_o.EpisodeMetrics(reset_obs(o, i), 2.5)
    rec = ev.records()
    assert len(rec) == len(expected) > 0
    got = {}
    for row in rec:
        got.setdefault(int(row[0]), []).append(row)
    for i, s, st in expected:
        row = got[i].pop(0)
        assert int(row[7]) == st
        _cmp_summary(row, s, st, i)


def _run_tracker(dev, fused, groups, native_groups=False, e=64, steps=70):
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import EvalTracker
    vec = VecSwarm(e, {"num_drones": 64, "max_steps": 30}, device=dev, auto_reset=True, seed=17, with_infos=True,
                   groups=groups)
    vec.reset()
    ev = EvalTracker(vec, capacity=8192, fused=fused)
    assert ev.fused == fused
    ev.begin()
    g = torch.Generator(device=dev).manual_seed(23)
    for _ in range(steps):
        a = torch.rand((e, 64, 3), device=dev, generator=g) * 2 - 1
        if native_groups:  # bench.py's launch: one swarm_step_groups call, group streams, no joins
            vec.fork_groups()
            vec.step_groups(a)
            vec.join()
        else:
            vec.step(a)
        ev.update()
    assert vec.kernel_name() == "swarm_step64_once<32, 4>"
    return ev.records()


@pytest.mark.parametrize("groups,native", [(1, False), (2, False), (2, True), (3, True)])
def test_fused_eval_equals_unfused(dev, groups, native):
    """SWARM_EVAL_STEP_FUSED (the step accumulates reward / steps / votes / path length in its
    write-back, swarm_eval_update only the formation error): the same records, bit for bit, as
    the unfused update at the headline shape (N = 64, swarm_step64_once), with env groups too."""
    a = _run_tracker(dev, True, groups, native)
    b = _run_tracker(dev, False, 1)
    assert len(a) > 64 and a.shape == b.shape
    assert np.array_equal(a, b, equal_nan=True)


def _tracker_session(dev, fused, *, reset_observe=False, env_cfg=False, e=64, steps=40):
    """Steps with a tracker, then (optionally) vec.reset() + vec.observe() + begin() or a per-env
    config that moves the step off step64, then more steps: the records."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import EvalTracker
    vec = VecSwarm(e, {"num_drones": 64, "max_steps": 25}, device=dev, auto_reset=True, seed=5, with_infos=True,
                   groups=2)
    vec.reset()
    ev = EvalTracker(vec, capacity=8192, fused=fused)
    ev.begin()
    g = torch.Generator(device=dev).manual_seed(29)
    for k in range(2 * steps):
        if k == steps and reset_observe:
            vec.reset()
            vec.observe()
            ev.begin()
        if k == steps and env_cfg:
            vec.set_env_config(world_size=20.0)  # the batch value: same results as no record
            assert not ev.fused
        vec.step(torch.rand((e, 64, 3), device=dev, generator=g) * 2 - 1)
        ev.update()
    return ev.records()


def test_fused_tracker_then_reset_observe(dev):
    """a fused tracker attached, then vec.reset(), vec.observe() and begin()
    (the out struct with out.eval goes to the reset / observe launches too), then more steps — the
    same records as an unfused tracker over the same calls."""
    a = _tracker_session(dev, True, reset_observe=True)
    b = _tracker_session(dev, False, reset_observe=True)
    assert len(a) > 64 and np.array_equal(a, b, equal_nan=True)


def test_set_env_config_detaches_fused_tracker(dev):
    """per-env records move the step to the generic kernel; the fused tracker goes
    back to unfused updates instead of every later step failing."""
    a = _tracker_session(dev, True, env_cfg=True)
    b = _tracker_session(dev, False, env_cfg=True)
    assert len(a) > 64 and np.array_equal(a, b, equal_nan=True)


def test_second_fused_tracker_takes_over(dev):
    """a second fused tracker takes the steps over and the first goes back to
    unfused updates (both keep recording); the first one's detach() does not unhook the second."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import EvalTracker
    e = 64
    vec = VecSwarm(e, {"num_drones": 64, "max_steps": 25}, device=dev, auto_reset=True, seed=5, with_infos=True)
    vec.reset()
    ev1 = EvalTracker(vec, capacity=8192)
    assert ev1.fused
    ev2 = EvalTracker(vec, capacity=8192)
    assert ev2.fused and not ev1.fused and vec._eval_owner is ev2
    ev1.begin()
    ev2.begin()
    g = torch.Generator(device=dev).manual_seed(31)
    for k in range(60):
        if k == 20:
            ev1.detach()  # not the owner: a no-op for the steps
            assert ev2.fused and vec._gout[0].eval is not None
        vec.step(torch.rand((e, 64, 3), device=dev, generator=g) * 2 - 1)
        ev1.update()
        ev2.update()
    a, b = ev1.records(), ev2.records()
    assert len(a) > 32 and np.array_equal(a, b, equal_nan=True)


def test_record_blocks_only_for_live_segments(dev):
    """E < 64 envs write min(E, 64) record segments: only those blocks are allocated (ADVICE r03:
    E = 1 at the default capacity took 64 blocks, ~302 MB), also at an env_offset that wraps
    the segment ring."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import EvalTracker
    vec = VecSwarm(3, {"num_drones": 4, "max_steps": 5}, device=dev, auto_reset=True, with_infos=True,
                   env_offset=126)  # global envs 126, 127, 128: segments 62, 63, 0
    vec.reset()
    ev = EvalTracker(vec, capacity=90)
    assert ev.segments == 3 and ev.seg_base == 62 and ev.records_buf.shape[0] == 90
    ev.begin()
    for _ in range(26):
        vec.step(torch.zeros((3, 4, 3), device=dev))
        ev.update()
    rec = ev.records()
    assert sorted(set(rec[:, 0].astype(int))) == [126, 127, 128]
    assert len(rec) >= 15 and np.all(rec[:, 7] <= 5)  # episodes end by the 5-step time limit or earlier


def test_fused_eval_needs_step64(dev):
    """out.eval on a launch other than the kinematic step64 one is refused (SWARM_EINVAL)."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import EvalTracker
    vec = VecSwarm(8, {"num_drones": 16}, device=dev, auto_reset=True, with_infos=True)
    vec.reset()
    assert EvalTracker(vec).fused is False  # auto: not the step64 kernel
    ev = EvalTracker(vec, fused=True)
    with pytest.raises(ValueError, match="step64"):
        vec.step(torch.zeros((8, 16, 3), device=dev))
    ev.detach()
    vec.step(torch.zeros((8, 16, 3), device=dev))


def test_curriculum_runner_stages(dev):
    from swarm_marl_amd.curriculum import CurriculumRunner
    from tests.test_eval_cpu import STAGES
    run = CurriculumRunner(STAGES, 32, base_seed=3, device=dev)
    seen = []
    while not run.done:
        v = run.vec
        seen.append((v.num_drones, int(v.cfg.num_obstacles)))
        g = torch.Generator(device=dev).manual_seed(run.index)
        while not run.ready():
            for _ in range(40):
                run.step(torch.rand((32, v.num_drones, 3), device=dev, generator=g) * 2 - 1)
            run.end_iteration()
        m = run.window_metrics()
        assert m["episodes"] > 0 and 0.0 <= m["success_rate"] <= 1.0
        run.advance()
    assert seen == [(3, 0), (5, 4)]


EVAL1_FIXTURES = sorted(p.name for p in GOLDEN.glob("eval1_*.npz"))


@pytest.mark.parametrize("name", EVAL1_FIXTURES)
def test_single_agent_eval_replays_reference_episodes(dev, name):
    """evaluate_protocol.py:193-234 over the reference SingleDroneEnv (eval1_*.npz, made by the
    reference's own function): each recorded episode is one single-drone env of a VecSwarm from
    its recorded reset state and actions, stepped by the HIP kernel and measured by
    swarm_eval_single_update.  The fixtures hold goal-reached, collision (SR = CFR = 0) and
    time-limit (NaN TTG) episodes; the terminal step's info and position count."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import SingleAgentEvalTracker
    d = np.load(GOLDEN / name)
    cfg = dict(json.loads(str(d["config"])), neighbor_k=0)
    lens = d["lengths"]
    e = len(lens)
    vec = VecSwarm(e, cfg, num_drones=1, device=dev, auto_reset=False, with_infos=True, seed=77)
    vec.set_state(pos=d["reset_pos"].reshape(e, 1, 3), vel=np.zeros((e, 1, 3), np.float32), goal=d["reset_goal"],
                  obstacles=d["reset_obst"], active=np.ones((e, 1), bool), step_count=np.zeros(e, np.int32))
    vec.observe()
    ev = SingleAgentEvalTracker(vec, capacity=4096)
    ev.begin()
    acts = torch.as_tensor(d["actions"], device=dev)  # [episodes, T, 3]
    for t in range(int(lens.max())):
        a = acts[:, t].reshape(e, 1, 3).contiguous()
        vec.step(a)
        ev.update()  # finished envs are reset on the device and start new (unrecorded) episodes
    rec = ev.records()
    first = {}
    for row in rec:  # completion order: the first record of each env is the recorded episode
        first.setdefault(int(row[0]), row)
    assert sorted(first) == list(range(e))
    sm = d["summaries"]
    for k in range(e):
        row = first[k]
        assert int(row[7]) == int(lens[k]), (name, k)
        _cmp_summary(row, sm[k], int(lens[k]), (name, k))
    got = [first[k] for k in range(e)]
    from swarm_marl_amd.eval_metrics import aggregate_records
    agg, ref = aggregate_records(np.stack(got)), json.loads(str(d["aggregate"]))
    for key in ("success_rate", "collision_free_rate"):
        assert agg[key] == ref[key], key
    assert (math.isnan(agg["mean_time_to_goal"]) and math.isnan(ref["mean_time_to_goal"])) or \
        agg["mean_time_to_goal"] == ref["mean_time_to_goal"]
    assert agg["path_efficiency"] == pytest.approx(ref["path_efficiency"], rel=1e-9)
    assert (sm[:, 0] == 0).any() or (sm[:, 1] == 0).any()  # the failure branches are exercised


def test_single_agent_eval_rejects_swarm_batches(dev):
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.eval_metrics import SingleAgentEvalTracker
    with pytest.raises(ValueError):
        SingleAgentEvalTracker(VecSwarm(4, {"num_drones": 3}, device=dev, auto_reset=False, with_infos=True))
    with pytest.raises(ValueError):
        SingleAgentEvalTracker(VecSwarm(4, {"neighbor_k": 0}, num_drones=1, device=dev, auto_reset=True,
                                        with_infos=True))
