"""Curriculum stages on the device engine (configs/curriculum_v1.yaml).

The reference's curriculum (scripts/train_curriculum.py:159-233) walks a list of stages, each
an `env_config` (num_drones, num_obstacles, max_steps, world_size) trained for
`train_iterations` with `seed = base_seed + stage_index`; the YAML also states promotion
criteria over a rolling window of episodes (min success rate, min collision-free rate, max mean
time to goal; `promotion_window_episodes`), which the reference script records but does not
enforce.  Here a stage is a VecSwarm of E envs built from that env_config (stages change N and
M, i.e. the tensor shapes, so each stage is its own batch) with an EvalTracker; the window
metrics come from the device eval records and `advance()` moves on by iteration count, or by
the criteria when asked to.

Stages that share N (stages 1-2 of curriculum_v1 are both N = 3) can also run side by side in ONE
batch: `mixed_stage_batch` gives each env its stage's num_obstacles / max_steps / world_size as
per-env parameters (swarm_env_cfg_t), so a curriculum can keep a replay fraction of earlier
stages without a second launch.
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Any

import numpy as np

from .eval_metrics import EvalTracker, aggregate_records
from .vec_env import VecSwarm


def load_curriculum(path: str | Path) -> dict[str, Any]:
    """The curriculum mapping from a YAML / JSON file (yaml.safe_load: data only)."""
    p = Path(path)
    text = p.read_text(encoding="utf-8")
    if p.suffix.lower() == ".json":
        import json
        cfg = json.loads(text)
    else:
        import yaml
        cfg = yaml.safe_load(text)
    stages = cfg.get("stages") if isinstance(cfg, dict) else None
    if not isinstance(stages, list) or not stages:
        raise ValueError(f"no stages in curriculum config {p}")
    for i, st in enumerate(stages):
        if not isinstance(st, dict):
            raise ValueError(f"stage index {i} is not a mapping")
    return cfg


def stage_env_config(cfg: dict, index: int, base_seed: int = 0) -> dict[str, Any]:
    """env_config of stage `index` with the reference's per-stage seed (train_curriculum.py:187-188)."""
    env_cfg = dict(cfg["stages"][index].get("env_config", {}))
    env_cfg["seed"] = int(base_seed + index)
    return env_cfg


STAGE_PARAMS = ("world_size", "dt", "max_speed", "max_accel", "obstacle_radius", "max_steps", "num_obstacles")


def mixed_stage_batch(cfg: dict, stage_of_env, *, base_seed: int = 0, seed: int | None = None, device=None,
                      **vec_kw):
    """One VecSwarm whose env e runs stage stage_of_env[e]'s env_config (stages must share
    num_drones and the env_config keys other than STAGE_PARAMS).  Returns (vec, overrides): the
    batch holds max(num_obstacles) obstacle slots and every stage parameter as a per-env value;
    `overrides` maps each parameter to its [E] numpy array."""
    stages = np.asarray(stage_of_env, dtype=np.int64)
    if stages.ndim != 1 or len(stages) == 0:
        raise ValueError("stage_of_env must be a non-empty 1-D sequence of stage indices")
    used = sorted(set(int(i) for i in stages))
    if used[0] < 0 or used[-1] >= len(cfg["stages"]):
        raise ValueError(f"stage index out of range [0, {len(cfg['stages'])})")
    env_cfgs = {i: stage_env_config(cfg, i, base_seed) for i in used}
    n_set = {int(c.get("num_drones", 3)) for c in env_cfgs.values()}
    if len(n_set) != 1:
        raise ValueError(f"stages {used} differ in num_drones {sorted(n_set)}: they cannot share a batch")
    rest = [{k: v for k, v in c.items() if k not in STAGE_PARAMS + ("seed",)} for c in env_cfgs.values()]
    if any(r != rest[0] for r in rest):
        raise ValueError("stages differ in fields other than " + ", ".join(STAGE_PARAMS))
    from .envs.common import DroneEnvConfig
    batch = dict(rest[0])
    batch["num_obstacles"] = max(int(c.get("num_obstacles", DroneEnvConfig.num_obstacles)) for c in env_cfgs.values())
    defaults = DroneEnvConfig()
    over = {}
    for k in STAGE_PARAMS:
        vals = [env_cfgs[int(i)].get(k, getattr(defaults, k)) for i in stages]
        over[k] = np.asarray(vals, dtype=np.int32 if k in ("max_steps", "num_obstacles") else np.float64)
    vec = VecSwarm(len(stages), batch, device=device, auto_reset=True,
                   seed=int(base_seed if seed is None else seed), **vec_kw)
    vec.set_env_config(**over)
    return vec, over


def criteria_met(metrics: dict, criteria: dict | None) -> bool:
    """The YAML's promotion_criteria against aggregated metrics (a NaN time-to-goal fails a
    max_mean_time_to_goal bound; no criteria = met)."""
    if not criteria:
        return True
    if "min_success_rate" in criteria and not metrics["success_rate"] >= float(criteria["min_success_rate"]):
        return False
    if "min_collision_free_rate" in criteria and \
            not metrics["collision_free_rate"] >= float(criteria["min_collision_free_rate"]):
        return False
    if "max_mean_time_to_goal" in criteria:
        ttg = metrics["mean_time_to_goal"]
        if math.isnan(ttg) or ttg > float(criteria["max_mean_time_to_goal"]):
            return False
    return True


class CurriculumRunner:
    """Current stage's VecSwarm (auto-reset, infos) + EvalTracker; `advance()` builds the next."""

    def __init__(self, cfg: dict, num_envs: int, *, base_seed: int = 0, device=None, **vec_kw):
        self.cfg = cfg
        self.num_envs = int(num_envs)
        self.base_seed = int(base_seed)
        self.device = device
        self.vec_kw = vec_kw
        self.window = int(cfg.get("promotion_window_episodes", 100))
        self.index = -1
        self.iterations = 0
        self.vec: VecSwarm | None = None
        self.tracker: EvalTracker | None = None
        self._build(0)

    @property
    def stage(self) -> dict:
        return self.cfg["stages"][self.index]

    @property
    def done(self) -> bool:
        return self.index >= len(self.cfg["stages"])

    def _build(self, index: int) -> None:
        self.index = index
        self.iterations = 0
        if self.done:
            self.vec = self.tracker = None
            return
        env_cfg = stage_env_config(self.cfg, index, self.base_seed)
        self.vec = VecSwarm(self.num_envs, env_cfg, device=self.device, auto_reset=True,
                            seed=env_cfg["seed"], with_infos=True, **self.vec_kw)
        self.vec.reset()
        self.tracker = EvalTracker(self.vec)
        self.tracker.begin()

    def step(self, actions, action_mask=None):
        out = self.vec.step(actions, action_mask)
        self.tracker.update()
        return out

    def end_iteration(self) -> None:
        self.iterations += 1

    def window_metrics(self) -> dict:
        rec = self.tracker.records()
        return aggregate_records(rec[-self.window:])

    def ready(self, use_criteria: bool = False) -> bool:
        """Stage finished: its train_iterations are done (the reference's rule), or — with
        use_criteria — a full window of episodes meets promotion_criteria."""
        if use_criteria:
            m = self.window_metrics()
            return m["episodes"] >= self.window and criteria_met(m, self.stage.get("promotion_criteria"))
        return self.iterations >= int(self.stage.get("train_iterations", 50))

    def advance(self) -> bool:
        """Move to the next stage; False once past the last."""
        self._build(self.index + 1)
        return not self.done
