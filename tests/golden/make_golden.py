"""Generate golden fixtures for the swarm step/reset hot path from the REFERENCE.

Run only in the build container (it reads /root/reference, which never travels to the
GPU box):  python tests/golden/make_golden.py

The reference `DroneSwarmEnv` / `SingleDroneEnv` (src/swarm_marl/envs/drone_swarm_env.py,
single_drone_env.py) import gymnasium only for `spaces.Box` / `gym.Env`; gymnasium is not
installed here, so a minimal stand-in module is injected into sys.modules before the import
(SURVEY.md §8c).  ray is absent; the reference's own stub MultiAgentEnv is used
(drone_swarm_env.py:8-12).

Each fixture is an .npz of inputs (pre-step state, actions) and outputs (obs, rewards,
terminated/truncated incl. "__all__", infos, post-step state) recorded step by step.
These are DATA only; no reference source is copied.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def _install_gymnasium_shim() -> None:
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    class Env:
        def reset(self, *, seed=None, options=None):
            return None

    spaces.Box = Box
    gym.spaces = spaces
    gym.Env = Env
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces


_install_gymnasium_shim()
sys.path.insert(0, REF_SRC)
from swarm_marl.envs.drone_swarm_env import DroneSwarmEnv  # noqa: E402
from swarm_marl.envs.single_drone_env import SingleDroneEnv  # noqa: E402


def _snapshot(env):
    return dict(
        pos=env.positions.copy(),
        vel=env.velocities.copy(),
        goal=env.goal.copy(),
        obst=env.obstacles.copy(),
        active=np.array([a in env.agents for a in env.agent_ids], dtype=bool),
        step=np.int32(env.step_count),
    )


class Recorder:
    """Collects per-step records of a DroneSwarmEnv rollout into stacked arrays."""

    def __init__(self, env):
        self.env = env
        self.rows: list[dict] = []

    def step(self, actions: np.ndarray, present: np.ndarray, extra: dict | None = None):
        env = self.env
        n = env.num_drones
        pre = _snapshot(env)
        action_dict = {}
        for i, aid in enumerate(env.agent_ids):
            if present[i]:
                action_dict[aid] = actions[i].copy()
        if extra:
            action_dict.update(extra)
        obs, rew, term, trunc, infos = env.step(action_dict)
        post = _snapshot(env)
        d = env._obs_dim
        row = dict(
            pre_pos=pre["pos"], pre_vel=pre["vel"], pre_goal=pre["goal"], pre_obst=pre["obst"],
            pre_active=pre["active"], pre_step=pre["step"],
            actions=np.where(present[:, None], actions, 0).astype(np.float32),
            action_present=present.copy(),
            out_obs=np.zeros((n, d), np.float32), obs_present=np.zeros(n, bool),
            rew=np.zeros(n, np.float64), rew_present=np.zeros(n, bool),
            term=np.zeros(n, bool), term_present=np.zeros(n, bool),
            trunc=np.zeros(n, bool),
            term_all=bool(term["__all__"]), trunc_all=bool(trunc["__all__"]),
            info_dist=np.zeros(n, np.float64), info_reached=np.zeros(n, bool),
            info_collision=np.zeros(n, bool), info_present=np.zeros(n, bool),
            global_state=np.concatenate([post["pos"].reshape(-1), post["vel"].reshape(-1),
                                         post["goal"]]).astype(np.float32),
            post_pos=post["pos"], post_vel=post["vel"], post_active=post["active"],
            post_step=post["step"],
        )
        for i, aid in enumerate(env.agent_ids):
            if aid in obs:
                row["out_obs"][i] = obs[aid]
                row["obs_present"][i] = True
            if aid in rew:
                assert isinstance(rew[aid], float)
                row["rew"][i] = rew[aid]
                row["rew_present"][i] = True
            if aid in term:
                row["term"][i] = term[aid]
                row["trunc"][i] = trunc[aid]
                row["term_present"][i] = True
            if aid in infos:
                inf = infos[aid]
                row["info_dist"][i] = inf["distance_to_goal"]
                row["info_reached"][i] = inf["reached_goal"]
                row["info_collision"][i] = inf["collision"]
                row["info_present"][i] = True
                assert np.array_equal(inf["global_state"], row["global_state"])
        self.rows.append(row)
        return term["__all__"] or trunc["__all__"]

    def save(self, name: str, cfg: dict, meta: dict | None = None):
        out = {k: np.stack([r[k] for r in self.rows]) for k in self.rows[0]}
        out["config"] = np.array(json.dumps(cfg))
        out["meta"] = np.array(json.dumps(meta or {}))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(f"{name}: {len(self.rows)} steps -> {os.path.getsize(path)} B")


def _record_reset(env, seed):
    obs, infos = env.reset(seed=seed)
    n, d = env.num_drones, env._obs_dim
    o = np.stack([obs[a] for a in env.agent_ids]) if n else np.zeros((0, d), np.float32)
    dist = np.array([infos[a]["distance_to_goal"] for a in env.agent_ids], np.float64)
    gs = infos[env.agent_ids[0]]["global_state"] if n else np.zeros(3, np.float32)
    return dict(pos=env.positions.copy(), vel=env.velocities.copy(), goal=env.goal.copy(),
                obst=env.obstacles.copy(), obs=o, dist=dist, global_state=gs)


def rollout_case(name, cfg, steps, action_seed, *, missing_prob=0.0, scale=1.0,
                 reset_seeds=None, max_resets=1000):
    """Seeded rollout with auto-reset on episode end; every reset gets a recorded seed."""
    env = DroneSwarmEnv(cfg)
    rng = np.random.default_rng(action_seed)
    rec = Recorder(env)
    seeds = list(reset_seeds or [])
    used = []
    s0 = seeds.pop(0) if seeds else None
    env.reset(seed=s0)
    used.append(-1 if s0 is None else s0)
    for _ in range(steps):
        acts = (rng.uniform(-1, 1, size=(env.num_drones, 3)) * scale).astype(np.float32)
        present = rng.uniform(size=env.num_drones) >= missing_prob
        done = rec.step(acts, present)
        if done and len(used) < max_resets:
            s = seeds.pop(0) if seeds else None
            env.reset(seed=s)
            used.append(-1 if s is None else s)
    rec.save(name, cfg, {"action_seed": action_seed, "reset_seeds": used})


def reset_case(name, cfg, seeds):
    env = DroneSwarmEnv(cfg)
    rows = [_record_reset(env, s) for s in seeds]
    # also: reset() with no seed continues the cfg.seed stream (drone_swarm_env.py:66-67)
    env2 = DroneSwarmEnv(cfg)
    rows_cont = [_record_reset(env2, None) for _ in range(3)]
    out = {f"seeded_{k}": np.stack([r[k] for r in rows]) for k in rows[0]}
    out.update({f"cont_{k}": np.stack([r[k] for r in rows_cont]) for k in rows_cont[0]})
    out["seeds"] = np.array(seeds, np.int64)
    out["config"] = np.array(json.dumps(cfg))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(seeds)} seeds -> {os.path.getsize(path)} B")


def injected_case(name, cfg, build, steps, action_fn):
    """Deterministic state injection (public attributes, drone_swarm_env.py:59-63)."""
    env = DroneSwarmEnv(cfg)
    env.reset(seed=cfg.get("seed", 0))
    build(env)
    rec = Recorder(env)
    for t in range(steps):
        acts, present, extra = action_fn(env, t)
        done = rec.step(acts, present, extra)
        if done:
            # one extra call after the episode ended: returns {"__all__": True}
            rec.step(acts, present, extra)
            break
    rec.save(name, cfg)


def _zeros(env, t):
    return np.zeros((env.num_drones, 3), np.float32), np.ones(env.num_drones, bool), None


def main():
    # --- config 1: N=4, E=1, 200 steps (BASELINE.json configs[0])
    rollout_case("rollout_n4", {"num_drones": 4, "seed": 123}, 200, 1000,
                 reset_seeds=list(range(100, 140)))
    # N=4 with missing actions and out-of-range actions (action clip, drone_swarm_env.py:104-106)
    rollout_case("rollout_n4_missing", {"num_drones": 4, "seed": 5, "max_steps": 60}, 150, 1001,
                 missing_prob=0.3, scale=2.5, reset_seeds=list(range(200, 260)))
    # N=16 and N=64: default radii (episodes end fast) and no-termination variant (radii 0)
    rollout_case("rollout_n16", {"num_drones": 16, "seed": 11}, 40, 1002,
                 reset_seeds=list(range(300, 400)))
    rollout_case("rollout_n16_noterm", {"num_drones": 16, "seed": 12, "collision_radius": 0.0,
                                         "obstacle_radius": 0.0, "goal_radius": 0.0}, 40, 1003,
                 scale=1.5, reset_seeds=[301])
    rollout_case("rollout_n64", {"num_drones": 64, "seed": 13}, 12, 1004,
                 reset_seeds=list(range(400, 420)))
    rollout_case("rollout_n64_noterm", {"num_drones": 64, "seed": 14, "collision_radius": 0.0,
                                         "obstacle_radius": 0.0, "goal_radius": 0.0}, 8, 1005,
                 reset_seeds=[401])
    # K > N-1 zero padding (N=3, K=3 default) and odd configs
    rollout_case("rollout_n3_k3", {"num_drones": 3, "seed": 21, "max_steps": 25}, 80, 1006,
                 reset_seeds=list(range(500, 540)))
    rollout_case("rollout_n1", {"num_drones": 1, "seed": 22, "max_steps": 30}, 70, 1007,
                 reset_seeds=list(range(600, 640)))
    rollout_case("rollout_n5_k6_s10_m6", {"num_drones": 5, "seed": 23, "neighbor_k": 6,
                                          "sensed_obstacles": 10, "num_obstacles": 6,
                                          "max_steps": 30}, 60, 1008,
                 reset_seeds=list(range(700, 740)))
    rollout_case("rollout_n6_k0_m0", {"num_drones": 6, "seed": 24, "neighbor_k": 0,
                                      "num_obstacles": 0, "sensed_obstacles": 2,
                                      "max_steps": 20}, 50, 1009,
                 reset_seeds=list(range(800, 840)))
    rollout_case("rollout_n8_custom", {"num_drones": 8, "seed": 25, "world_size": 12.0,
                                       "dt": 0.05, "max_speed": 1.5, "max_accel": 5.0,
                                       "desired_spacing": 1.7, "reward_formation_scale": 0.4,
                                       "reward_progress_scale": 3.0, "reward_goal": 10.0,
                                       "reward_collision": -7.0, "collision_radius": 0.2,
                                       "obstacle_radius": 0.3, "goal_radius": 1.5,
                                       "max_steps": 40}, 80, 1010,
                 scale=3.0, reset_seeds=list(range(900, 960)))

    # --- reset draws (drone_swarm_env.py:65-90)
    reset_case("reset_n4", {"num_drones": 4, "seed": 123}, [0, 1, 2, 123, 2**31 - 1])
    reset_case("reset_n64", {"num_drones": 64, "seed": 7}, [0, 99])

    # --- injected edge cases
    def goal_reach(env):
        env.goal = np.array([1.0, 1.0, 1.0], np.float32)
        env.obstacles[:] = np.array([9.0, -9.0, 9.0], np.float32)
        env.positions = np.array([[1.0, 1.0, 1.85], [-5, -5, -5], [5, 5, -5], [-5, 5, 5]],
                                 np.float32)
        env.velocities = np.array([[0, 0, -1.0], [0, 0, 0], [0, 0, 0], [0, 0, 0]], np.float32)

    def goal_reach_acts(env, t):
        a = np.zeros((4, 3), np.float32)
        a[1:] = [0.3, -0.2, 0.1]
        return a, np.ones(4, bool), None
    injected_case("edge_goal_reach", {"num_drones": 4, "seed": 1}, goal_reach, 6, goal_reach_acts)

    def all_reach(env):
        env.goal = np.array([0.0, 0.0, 0.0], np.float32)
        env.obstacles[:] = np.array([9.0, -9.0, 9.0], np.float32)
        env.positions = np.array([[0.5, 0, 0], [-0.5, 0, 0.2]], np.float32)
        env.velocities[:] = 0
    injected_case("edge_all_reached", {"num_drones": 2, "seed": 2, "collision_radius": 0.1},
                  all_reach, 3, _zeros)

    def pair_collide(env):
        env.obstacles[:] = np.array([9.0, -9.0, 9.0], np.float32)
        env.positions = np.array([[0, 0, 0], [1.2, 0, 0], [-5, 3, 2], [6, 6, 6]], np.float32)
        env.velocities = np.array([[1.0, 0, 0], [-1.0, 0, 0], [0, 0, 0], [0, 0, 0]], np.float32)
        env.goal = np.array([-8.0, 8.0, 0.0], np.float32)
    injected_case("edge_pair_collision", {"num_drones": 4, "seed": 3}, pair_collide, 4, _zeros)

    def obst_collide(env):
        env.obstacles[:] = np.array([9.0, -9.0, 9.0], np.float32)
        env.obstacles[2] = np.array([2.0, 2.0, 2.0], np.float32)
        env.positions = np.array([[2.0, 2.0, 3.45], [-5, -5, -5], [5, 5, -5]], np.float32)
        env.velocities = np.array([[0, 0, -1.0], [0, 0, 0], [0, 0, 0]], np.float32)
        env.goal = np.array([-8.0, 8.0, 0.0], np.float32)
    injected_case("edge_obstacle_collision", {"num_drones": 3, "seed": 4}, obst_collide, 4, _zeros)

    def wall(env):
        env.obstacles[:] = np.array([0.0, 0.0, -9.0], np.float32)
        env.positions = np.array([[9.9, -9.95, 9.8], [-9.9, 9.9, -9.9], [0, 0, 0]], np.float32)
        env.velocities = np.array([[3.9, -3.9, 1.0], [-3.0, 3.0, -3.0], [0, 0, 0]], np.float32)
        env.goal = np.array([9.0, 9.0, 9.0], np.float32)

    def wall_acts(env, t):
        a = np.array([[1.5, -3.0, 1.0], [-1.0, 1.0, -0.7], [0.9, 0.9, 0.9]], np.float32)
        return a, np.ones(3, bool), None
    injected_case("edge_wall_speed_clip", {"num_drones": 3, "seed": 5, "max_steps": 30}, wall, 12,
                  wall_acts)

    def tl_build(env):
        env.obstacles[:] = np.array([9.5, 9.5, 9.5], np.float32)
        env.positions = np.array([[-6, -6, -6], [6, -6, 6], [-6, 6, 6]], np.float32)
        env.velocities[:] = 0
        env.goal = np.array([0.0, 0.0, 0.0], np.float32)

    def tl_acts(env, t):
        a = np.full((3, 3), 0.01, np.float32)
        # unknown agent id is ignored by the swarm env (drone_swarm_env.py:103-104)
        return a, np.array([True, t % 2 == 0, True]), {"drone_99": np.ones(3, np.float32)}
    injected_case("edge_time_limit", {"num_drones": 3, "seed": 6, "max_steps": 5}, tl_build, 8,
                  tl_acts)

    def frozen(env):
        # drone 0 reaches its goal at step 1, stays frozen and visible as a neighbour
        env.goal = np.array([0.0, 0.0, 0.0], np.float32)
        env.obstacles[:] = np.array([9.0, 9.0, -9.0], np.float32)
        env.positions = np.array([[0.3, 0.0, 0.0], [2.0, 0, 0], [-2.5, 0.5, 0], [0, 3.5, 0.5],
                                  [0, -3, -1]], np.float32)
        env.velocities[:] = 0

    def frozen_acts(env, t):
        a = np.zeros((5, 3), np.float32)
        a[1] = [0.5, 0.5, 0.0]
        a[2] = [-0.3, 0.2, 0.4]
        a[3] = [0.1, -0.2, 0.2]
        a[4] = [0.2, 0.2, -0.2]
        return a, np.ones(5, bool), None
    injected_case("edge_frozen_neighbor", {"num_drones": 5, "seed": 7, "goal_radius": 0.5,
                                           "collision_radius": 0.3}, frozen, 10, frozen_acts)

    # --- SingleDroneEnv (single_drone_env.py:73-111): N=1, obs dim 9 + 4*M_s
    sd = SingleDroneEnv({"seed": 123, "max_steps": 50})
    rng = np.random.default_rng(2024)
    rows = []
    obs, info = sd.reset(seed=31)
    for t in range(120):
        a = rng.uniform(-1.4, 1.4, 3).astype(np.float32)
        pre = (sd.position.copy(), sd.velocity.copy(), sd.goal.copy(), sd.obstacles.copy(),
               np.int32(sd.step_count))
        o, r, te, tr, inf = sd.step(a)
        rows.append(dict(pre_pos=pre[0], pre_vel=pre[1], pre_goal=pre[2], pre_obst=pre[3],
                         pre_step=pre[4], actions=a, out_obs=o, rew=np.float64(r), term=te,
                         trunc=tr, info_dist=np.float64(inf["distance_to_goal"]),
                         post_pos=sd.position.copy(), post_vel=sd.velocity.copy()))
        if te or tr:
            sd.reset(seed=32 + t)
    out = {k: np.stack([np.asarray(r[k]) for r in rows]) for k in rows[0]}
    out["config"] = np.array(json.dumps({"seed": 123, "max_steps": 50}))
    np.savez_compressed(os.path.join(HERE, "single_drone.npz"), **out)
    print("single_drone:", len(rows))


if __name__ == "__main__":
    main()
