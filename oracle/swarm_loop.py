"""Per-agent loop restatement of the swarm step — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

BASELINE.md §5 variant (a): the same algorithmic structure as the reference env — one env at a
time, Python loops over agents and over agent pairs, one `np.linalg.norm` per 3-vector, an
`np.argsort` per observation — so its timing is a like-for-like stand-in for the reference
`DroneSwarmEnv.step()` on a host where the reference itself is absent (the GPU box).  Only
tests/ and bench.py's cpu_baseline leg import it; the product never does.

Behaviour follows src/swarm_marl/envs/drone_swarm_env.py:
  reset           :65-90   (host numpy draws: positions, goal, obstacles)
  step            :92-174  (integrate + _clip_speed :179-183, world clip :113-117,
                            _collision_mask :185-208, _formation_penalties :210-224, rewards,
                            terminated / truncated / "__all__")
  observation     :226-291 (_build_obs, K nearest neighbours, Ms nearest obstacles)
  global state    :293-302
It is pinned bit-exactly to the reference's own fixtures (tests/test_cpu_baselines.py).
Arrays and dicts are returned in the reference's shapes (obs per agent id, float rewards).
"""
from __future__ import annotations

import numpy as np

_DEFAULTS = dict(world_size=20.0, dt=0.1, max_steps=400, max_speed=4.0, max_accel=2.0,
                 collision_radius=0.5, goal_radius=0.8, num_obstacles=8, sensed_obstacles=4,
                 neighbor_k=3, obstacle_radius=0.8, desired_spacing=2.5,
                 reward_progress_scale=2.0, reward_goal=25.0, reward_collision=-25.0,
                 reward_formation_scale=0.15)


class LoopSwarm:
    """One swarm env stepped agent by agent (numpy float32 rows, Python floats for rewards)."""

    def __init__(self, num_drones: int = 3, seed: int = 0, **cfg):
        c = dict(_DEFAULTS)
        c.update(cfg)
        self.c = c
        self.n = int(num_drones)
        self.rng = np.random.default_rng(seed)
        self.ids = [f"drone_{i}" for i in range(self.n)]
        self.live: list[int] = list(range(self.n))
        self.pos = np.zeros((self.n, 3), np.float32)
        self.vel = np.zeros((self.n, 3), np.float32)
        self.goal = np.zeros(3, np.float32)
        self.obst = np.zeros((int(c["num_obstacles"]), 3), np.float32)
        self.t = 0

    # ---------------------------------------------------------------- episode start
    def reset(self, seed: int | None = None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        h = self.c["world_size"] / 2.0
        self.live = list(range(self.n))
        self.t = 0
        self.pos = self.rng.uniform(-h, h, size=(self.n, 3)).astype(np.float32)
        self.vel = np.zeros((self.n, 3), np.float32)
        self.goal = self.rng.uniform(-h, h, size=3).astype(np.float32)
        self.obst = self.rng.uniform(-h, h, size=(int(self.c["num_obstacles"]), 3)).astype(np.float32)
        gs = self.state_vector()
        obs = {self.ids[i]: self.observe(i) for i in range(self.n)}
        info = {self.ids[i]: {"distance_to_goal": self._goal_dist(i), "global_state": gs.copy()}
                for i in range(self.n)}
        return obs, info

    # ---------------------------------------------------------------- pieces
    def _goal_dist(self, i: int) -> float:
        return float(np.linalg.norm(self.goal - self.pos[i]))

    def state_vector(self) -> np.ndarray:
        return np.concatenate([self.pos.ravel(), self.vel.ravel(), self.goal.ravel()]).astype(np.float32)

    def _limit_speed(self, v: np.ndarray) -> np.ndarray:
        s = np.linalg.norm(v)
        vmax = self.c["max_speed"]
        return v if (s <= vmax or s < 1e-8) else (v / s) * vmax

    def _hits(self, live: list[int]) -> set[int]:
        hit: set[int] = set()
        if not live:
            return hit
        if len(self.obst):
            rel = self.pos[live][:, None, :] - self.obst[None, :, :]
            near = np.any(np.linalg.norm(rel, axis=2) <= self.c["collision_radius"] + self.c["obstacle_radius"],
                          axis=1)
            hit.update(i for i, h in zip(live, near) if h)
        lim = 2.0 * self.c["collision_radius"]
        for a in range(len(live)):
            for b in range(a + 1, len(live)):
                i, j = live[a], live[b]
                if np.linalg.norm(self.pos[i] - self.pos[j]) <= lim:
                    hit.add(i)
                    hit.add(j)
        return hit

    def _spacing_terms(self, live: list[int]) -> dict[int, float]:
        out = {i: 0.0 for i in live}
        if len(live) < 2:
            return out
        for i in live:
            d = [float(np.linalg.norm(self.pos[i] - self.pos[j])) for j in live if j != i]
            err = float(np.mean(np.abs(np.asarray(d) - self.c["desired_spacing"])))
            out[i] = -self.c["reward_formation_scale"] * err
        return out

    def observe(self, i: int) -> np.ndarray:
        own = self.pos[i]
        k, ms = int(self.c["neighbor_k"]), int(self.c["sensed_obstacles"])
        feats = [own, self.vel[i], self.goal - own]
        nb = np.zeros(4 * max(k, 0), np.float32)
        if self.n > 1 and k > 0:
            others = [j for j in range(self.n) if j != i]
            vecs = [self.pos[j] - own for j in others]
            dists = np.asarray([float(np.linalg.norm(v)) for v in vecs])
            for slot, o in enumerate(np.argsort(dists)[:k]):
                v = vecs[int(o)]
                nb[4 * slot:4 * slot + 4] = (float(v[0]), float(v[1]), float(v[2]), float(dists[int(o)]))
        feats.append(nb)
        ob = np.zeros(4 * max(ms, 0), np.float32)
        if len(self.obst) and ms > 0:
            rel = self.obst - own
            dist = np.linalg.norm(rel, axis=1)
            for slot, m in enumerate(np.argsort(dist)[:ms]):
                ob[4 * slot:4 * slot + 4] = (float(rel[m][0]), float(rel[m][1]), float(rel[m][2]), float(dist[m]))
        feats.append(ob)
        return np.concatenate(feats).astype(np.float32)

    # ---------------------------------------------------------------- step
    def step(self, actions: dict[str, np.ndarray]):
        live = list(self.live)
        if not live:
            return {}, {}, {"__all__": True}, {"__all__": False}, {}
        c = self.c
        before = {i: self._goal_dist(i) for i in live}
        for i in live:
            a = np.clip(np.asarray(actions.get(self.ids[i], np.zeros(3, np.float32)), np.float32).reshape(3),
                        -1.0, 1.0)
            self.vel[i] = self._limit_speed(self.vel[i] + (a * c["max_accel"]) * c["dt"])
            self.pos[i] = self.pos[i] + self.vel[i] * c["dt"]
        h = c["world_size"] / 2.0
        self.pos = np.clip(self.pos, -h, h)
        self.t += 1
        after = {i: self._goal_dist(i) for i in live}
        hit = self._hits(live)
        spacing = self._spacing_terms(live)
        crash = any(i in hit for i in live)
        timeout = self.t >= c["max_steps"]
        obs, rew, term, trunc, info, nxt = {}, {}, {}, {}, {}, []
        for i in live:
            aid = self.ids[i]
            at_goal = after[i] <= c["goal_radius"]
            r = (before[i] - after[i]) * c["reward_progress_scale"] + spacing.get(i, 0.0)
            if at_goal:
                r += c["reward_goal"]
            if i in hit:
                r += c["reward_collision"]
            rew[aid] = float(r)
            done = bool(at_goal or i in hit)
            term[aid] = done
            trunc[aid] = bool(timeout and not done)
            if not (done or timeout or crash):
                obs[aid] = self.observe(i)
                info[aid] = {"distance_to_goal": after[i], "reached_goal": bool(at_goal),
                             "collision": i in hit, "global_state": self.state_vector()}
                nxt.append(i)
        ended = (not nxt and not crash and not timeout) or crash
        term["__all__"] = bool(ended)
        trunc["__all__"] = bool(timeout and not ended)
        self.live = [] if (term["__all__"] or trunc["__all__"]) else nxt
        return obs, rew, term, trunc, info


def run_for(num_envs: int, num_drones: int, seconds: float, seed: int = 0) -> tuple[int, float]:
    """Step `num_envs` LoopSwarm envs round-robin with uniform(-1, 1) actions for about
    `seconds`, re-drawing an env's episode when it ends (the batched API's auto-reset).
    Returns (agent-steps, elapsed seconds); an agent-step is one reward entry (len(rewards))."""
    import time

    envs = [LoopSwarm(num_drones, seed=seed + k) for k in range(num_envs)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(1000 + seed)
    count, t0 = 0, time.perf_counter()
    while True:
        for e in envs:
            acts = rng.uniform(-1, 1, (num_drones, 3)).astype(np.float32)
            _, rew, term, trunc, _ = e.step({e.ids[i]: acts[i] for i in range(num_drones)})
            count += len(rew)
            if term["__all__"] or trunc["__all__"]:
                e.reset()
        el = time.perf_counter() - t0
        if el >= seconds:
            return count, el
