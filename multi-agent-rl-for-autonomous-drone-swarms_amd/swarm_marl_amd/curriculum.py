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
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Any

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
