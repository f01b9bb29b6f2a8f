"""Generate golden fixtures for the on-device eval metrics from the REFERENCE.

Run only in the build container (it reads /root/reference, which never travels to the GPU box):
    python tests/golden/make_eval_golden.py

The reference computes its evaluation metrics in scripts/evaluate_protocol.py:103-116 (formation
error), :237-331 (`_run_single_episode_multi_agent`: success, collision-free, time-to-goal,
formation error, path efficiency, episode reward) and :334-350 (`_aggregate`).  That script
imports RLlib, PyBullet and the training package at module level (none importable here), so
only the metric functions are taken from it: their definitions are selected from the script's
syntax tree and executed in a namespace holding numpy / math / statistics, then run against the
reference `DroneSwarmEnv` (imported with the gymnasium stand-in of make_golden.py) with a
stand-in `algo` whose `compute_single_action` returns recorded deterministic actions (goal-seeking
with noise, so that goals are reached and collisions happen).

Per episode the fixture holds the reset state, the actions as called (and which agents were
asked), and the reference's EpisodeSummary; per case the `_aggregate` dict.  DATA only.
"""
from __future__ import annotations

import ast
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import DroneSwarmEnv, SingleDroneEnv  # noqa: E402  (gymnasium stand-in + reference import)

EVAL_SCRIPT = "/root/reference/scripts/evaluate_protocol.py"
WANTED = ("EpisodeSummary", "_safe_std", "_distance", "_formation_error_from_positions",
          "_run_single_episode_multi_agent", "_run_single_episode_single_agent", "_aggregate")


def load_metric_functions() -> dict:
    tree = ast.parse(open(EVAL_SCRIPT).read())
    keep = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in WANTED]
    assert {n.name for n in keep} == set(WANTED), [n.name for n in keep]
    mod = ast.Module(body=keep, type_ignores=[])
    ns: dict = {}
    exec("import math\nimport numpy as np\nfrom dataclasses import dataclass\nfrom typing import Any\n"
         "from statistics import mean, pstdev\n", ns)
    ns["DroneSwarmEnv"] = DroneSwarmEnv
    ns["SingleDroneEnv"] = SingleDroneEnv
    exec(compile(mod, EVAL_SCRIPT, "exec"), ns)
    return ns


class RecordingAlgo:
    """compute_single_action stand-in: goal-seeking action plus noise (explore=False is ignored),
    every call recorded as (agent index, action) in call order."""

    def __init__(self, env, seed: int, noise: float):
        self.env, self.rng, self.noise = env, np.random.default_rng(seed), noise
        self.calls: list[tuple[int, np.ndarray]] = []

    def compute_single_action(self, obs, policy_id=None, explore=False):
        g = np.asarray(obs[6:9], np.float64)
        nrm = np.linalg.norm(g)
        a = (g / nrm if nrm > 1e-9 else np.zeros(3)) + self.rng.normal(0, self.noise, 3)
        a = np.clip(a, -1.0, 1.0).astype(np.float32)
        self.calls.append((len(self.calls), a))
        return a


def run_case(fns, name: str, cfg: dict, episodes: int, seed: int, noise: float) -> None:
    env = DroneSwarmEnv(dict(cfg))
    n = env.num_drones
    resets, actions, present, summaries = [], [], [], []
    orig_reset, orig_step = env.reset, env.step
    cur = {}

    def reset(*, seed=None, options=None):
        out = orig_reset(seed=seed, options=options)
        resets.append(dict(pos=env.positions.copy(), goal=env.goal.copy(), obst=env.obstacles.copy()))
        cur["acts"], cur["pres"] = [], []
        return out

    def step(action_dict):
        a = np.zeros((n, 3), np.float32)
        p = np.zeros(n, bool)
        for aid, v in action_dict.items():
            i = env.agent_id_to_index[aid]
            a[i], p[i] = np.asarray(v, np.float32), True
        cur["acts"].append(a)
        cur["pres"].append(p)
        return orig_step(action_dict)

    env.reset, env.step = reset, step
    algo = RecordingAlgo(env, seed, noise)
    for _ in range(episodes):
        s = fns["_run_single_episode_multi_agent"](algo, env)
        summaries.append([s.success, s.collision_free, s.time_to_goal, s.formation_error,
                          s.path_efficiency, s.episode_reward])
        actions.append(np.stack(cur["acts"]))
        present.append(np.stack(cur["pres"]))
    agg = fns["_aggregate"]([fns["EpisodeSummary"](*[type(f)(v) for f, v in zip((0, 0, 0.0, 0.0, 0.0, 0.0), row)])
                             for row in summaries])
    lens = np.array([len(a) for a in actions], np.int32)
    tmax = int(lens.max())
    act = np.zeros((episodes, tmax, n, 3), np.float32)
    pres = np.zeros((episodes, tmax, n), bool)
    for k in range(episodes):
        act[k, :lens[k]] = actions[k]
        pres[k, :lens[k]] = present[k]
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, config=json.dumps(cfg), lengths=lens, actions=act, present=pres,
                        reset_pos=np.stack([r["pos"] for r in resets]),
                        reset_goal=np.stack([r["goal"] for r in resets]),
                        reset_obst=np.stack([r["obst"] for r in resets]),
                        summaries=np.array(summaries, np.float64),
                        summary_fields=np.array(["success", "collision_free", "time_to_goal",
                                                 "formation_error", "path_efficiency", "episode_reward"]),
                        aggregate=json.dumps(agg))
    print(f"{name}: {episodes} episodes, lengths {lens.tolist()}, {os.path.getsize(path)} B, agg {agg}")


def run_case_single(fns, name: str, cfg: dict, episodes: int, seed: int, noise: float) -> None:
    """evaluate_protocol.py:193-234 `_run_single_episode_single_agent` over the reference
    SingleDroneEnv: unlike the swarm protocol it sees the terminal step's info (collision,
    reached_goal) and position, so SR = 0, CFR = 0 and NaN TTG all occur."""
    env = SingleDroneEnv(dict(cfg))
    resets, actions, summaries = [], [], []
    orig_reset, orig_step = env.reset, env.step
    cur = {}

    def reset(*, seed=None, options=None):
        out = orig_reset(seed=seed, options=options)
        resets.append(dict(pos=env.position.copy(), goal=env.goal.copy(), obst=env.obstacles.copy()))
        cur["acts"] = []
        return out

    def step(action):
        cur["acts"].append(np.asarray(action, np.float32).reshape(3))
        return orig_step(action)

    env.reset, env.step = reset, step
    algo = RecordingAlgo(env, seed, noise)
    for _ in range(episodes):
        s = fns["_run_single_episode_single_agent"](algo, env)
        summaries.append([s.success, s.collision_free, s.time_to_goal, s.formation_error,
                          s.path_efficiency, s.episode_reward])
        actions.append(np.stack(cur["acts"]))
    agg = fns["_aggregate"]([fns["EpisodeSummary"](*[type(f)(v) for f, v in zip((0, 0, 0.0, 0.0, 0.0, 0.0), row)])
                             for row in summaries])
    lens = np.array([len(a) for a in actions], np.int32)
    act = np.zeros((episodes, int(lens.max()), 3), np.float32)
    for k in range(episodes):
        act[k, :lens[k]] = actions[k]
    sm = np.array(summaries, np.float64)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, config=json.dumps(cfg), lengths=lens, actions=act,
                        reset_pos=np.stack([r["pos"] for r in resets]),
                        reset_goal=np.stack([r["goal"] for r in resets]),
                        reset_obst=np.stack([r["obst"] for r in resets]),
                        summaries=sm,
                        summary_fields=np.array(["success", "collision_free", "time_to_goal",
                                                 "formation_error", "path_efficiency", "episode_reward"]),
                        aggregate=json.dumps(agg))
    print(f"{name}: {episodes} episodes, lengths {lens.tolist()}, success {sm[:, 0].tolist()}, "
          f"collision_free {sm[:, 1].tolist()}, {os.path.getsize(path)} B, agg {agg}")


def main() -> None:
    fns = load_metric_functions()
    run_case(fns, "eval_n4", {"num_drones": 4, "seed": 11, "max_steps": 120}, 6, seed=1, noise=0.6)
    run_case(fns, "eval_n8", {"num_drones": 8, "seed": 12, "max_steps": 80, "num_obstacles": 4}, 6,
             seed=2, noise=0.3)
    run_case(fns, "eval_n3_obst0", {"num_drones": 3, "seed": 13, "max_steps": 200, "num_obstacles": 0}, 5,
             seed=3, noise=0.2)
    # single-agent protocol: goal reached, obstacle collisions and time-limit episodes
    run_case_single(fns, "eval1_obst", {"seed": 21, "max_steps": 60, "num_obstacles": 12, "obstacle_radius": 1.6},
                    12, seed=4, noise=0.35)
    run_case_single(fns, "eval1_tl", {"seed": 22, "max_steps": 18, "num_obstacles": 6}, 8, seed=5, noise=1.2)


if __name__ == "__main__":
    main()
