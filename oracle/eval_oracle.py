"""CPU restatement of the reference's evaluation metrics — TEST INFRASTRUCTURE ONLY.

Only tests/ (and nothing on the product path) may import this module.  It restates, from the
dict outputs of an env step loop, the per-episode summary of
/root/reference/scripts/evaluate_protocol.py:
  * :103-116  formation error of a set of positions (mean over agents of the mean |d_ij - d*|),
  * :237-331  `_run_single_episode_multi_agent`: success, collision-free, time-to-goal,
              formation error, path efficiency, episode reward,
  * :193-234  `_run_single_episode_single_agent` (SingleDroneEnv: the terminal step's info and
              position count; formation error 0),
  * :334-350  `_aggregate` over episodes,
including the reference's behaviour that an agent without an observation contributes neither a
collision nor a "not reached" vote: on the terminal step (no observations at all,
drone_swarm_env.py:154) the all-reached test passes vacuously.  Pinned by
tests/golden/eval_*.npz and eval1_*.npz (generated from the reference by
tests/golden/make_eval_golden.py).
"""
from __future__ import annotations

import math
from statistics import mean, pstdev

import numpy as np


def distance(a: np.ndarray, b: np.ndarray) -> float:
    """float(np.linalg.norm(a - b)) of float32 3-vectors (the sdot 1-D norm path)."""
    return float(np.linalg.norm(np.asarray(a, np.float32) - np.asarray(b, np.float32)))


def formation_error(positions: dict, spacing: float) -> float:
    keys = list(positions)
    if len(keys) <= 1:
        return 0.0
    per_agent = []
    for i, a in enumerate(keys):
        d = [distance(positions[a], positions[b]) for j, b in enumerate(keys) if j != i]
        per_agent.append(float(np.mean(np.abs(np.asarray(d) - spacing))))
    return float(np.mean(per_agent))


class EpisodeMetrics:
    """Accumulates one episode from its reset observations and step outputs."""

    def __init__(self, reset_obs: dict, spacing: float):
        self.spacing = float(spacing)
        self.ids = list(reset_obs)
        self.start, self.goal, self.last = {}, {}, {}
        self.traveled = {}
        for a, o in reset_obs.items():
            p = np.asarray(o[0:3], np.float32)
            self.start[a] = p.copy()
            self.goal[a] = p + np.asarray(o[6:9], np.float32)
            self.last[a] = p.copy()
            self.traveled[a] = 0.0
        self.reward = 0.0
        self.steps = 0
        self.collided = False
        self.reached_step = None
        self.fe = []

    def update(self, obs: dict, rewards: dict, terminated: dict, truncated: dict, infos: dict) -> bool:
        self.steps += 1
        self.reward += float(np.mean(list(rewards.values()))) if rewards else 0.0
        now = {}
        all_reached = True
        for a, o in obs.items():
            p = np.asarray(o[0:3], np.float32)
            self.traveled[a] += distance(self.last[a], p)
            self.last[a] = p
            now[a] = p
            info = infos.get(a, {})
            if info.get("collision", False):
                self.collided = True
            if not info.get("reached_goal", False):
                all_reached = False
        self.fe.append(formation_error(now, self.spacing))
        if all_reached and self.reached_step is None:
            self.reached_step = self.steps
        return bool(terminated.get("__all__", False) or truncated.get("__all__", False))

    def summary(self) -> tuple:
        pe = []
        for a in self.ids:
            straight = distance(self.start[a], self.goal[a])
            t = self.traveled[a]
            pe.append(straight / t if t > 1e-8 else 0.0)
        return (int((not self.collided) and self.reached_step is not None), int(not self.collided),
                float(self.reached_step) if self.reached_step is not None else math.nan,
                float(np.mean(self.fe)) if self.fe else 0.0, float(np.mean(pe)) if pe else 0.0,
                float(self.reward))


class SingleEpisodeMetrics:
    """evaluate_protocol.py:193-234 restated: one SingleDroneEnv episode from its reset
    observation and the (obs, reward, terminated, truncated, info) of every step."""

    def __init__(self, reset_obs):
        o = np.asarray(reset_obs, np.float32)
        self.start = o[0:3].copy()
        self.goal = self.start + o[6:9]  # float32: start + goal vector, as the reference
        self.last = self.start.copy()
        self.traveled = 0.0
        self.reward = 0.0
        self.steps = 0
        self.reached_step = None
        self.collided = False

    def update(self, obs, reward, terminated, truncated, info) -> bool:
        self.steps += 1
        self.reward += float(reward)
        p = np.asarray(obs, np.float32)[0:3]
        self.traveled += distance(self.last, p)
        self.last = p.copy()
        if bool(info.get("collision", False)):
            self.collided = True
        if bool(info.get("reached_goal", False)) and self.reached_step is None:
            self.reached_step = self.steps
        return bool(terminated or truncated)

    def summary(self) -> tuple:
        straight = distance(self.start, self.goal)
        pe = straight / self.traveled if self.traveled > 1e-8 else 0.0
        return (int((not self.collided) and self.reached_step is not None), int(not self.collided),
                float(self.reached_step) if self.reached_step is not None else math.nan, 0.0, float(pe),
                float(self.reward))


def single_drone_step(env, action):
    """SingleDroneEnv.step (single_drone_env.py:73-111) through the per-agent swarm restatement
    with one drone and no neighbours (oracle/swarm_loop.LoopSwarm, pinned to the reference
    fixtures, single_drone.npz included): same integrator, reward terms and flags; unlike the
    swarm dict API it returns the terminal step's observation and info."""
    i = 0
    _, rew, _, _, _ = env.step({env.ids[i]: action})
    after = env._goal_dist(i)
    at_goal = after <= env.c["goal_radius"]
    hit = i in env._hits([i])
    obs = env.observe(i)
    info = {"distance_to_goal": after, "reached_goal": bool(at_goal), "collision": bool(hit)}
    return obs, rew[env.ids[i]], bool(at_goal or hit), bool(env.t >= env.c["max_steps"]), info


def aggregate(summaries) -> dict:
    s = [x[0] for x in summaries]
    c = [x[1] for x in summaries]
    ttg = [x[2] for x in summaries if not math.isnan(x[2])]
    fe = [x[3] for x in summaries]
    pe = [x[4] for x in summaries]
    rw = [x[5] for x in summaries]
    return {"success_rate": float(mean(s)) if s else 0.0,
            "collision_free_rate": float(mean(c)) if c else 0.0,
            "mean_time_to_goal": float(mean(ttg)) if ttg else math.nan,
            "formation_error": float(mean(fe)) if fe else 0.0,
            "path_efficiency": float(mean(pe)) if pe else 0.0,
            "episode_reward_mean": float(mean(rw)) if rw else 0.0,
            "episode_reward_std": float(pstdev(rw)) if len(rw) > 1 else 0.0}
