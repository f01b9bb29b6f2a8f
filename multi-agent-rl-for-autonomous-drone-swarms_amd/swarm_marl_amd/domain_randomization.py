"""Per-episode domain randomisation on the device.

The reference ships configs/domain_randomization_v1.yaml (`enabled: false`, `apply_on_reset:
true`): per-episode scale factors for dynamics, actuation, sensing and environment parameters,
plus an out-of-distribution evaluation profile.  No reference code reads it,
so there is no reference behaviour to match beyond the file's own statement: "randomize dynamics
and sensing per episode reset".  This module applies the entries that map onto the swarm env's
parameters, as per-env parameter records (swarm_env_cfg_t), entirely on the device:

    dynamics.max_accel_scale        -> max_accel       = base * U(min, max)
    dynamics.max_speed_scale        -> max_speed
    dynamics.dt_scale               -> dt              (kinematic integrator only)
    environment.obstacle_radius_scale -> obstacle_radius
    environment.world_size_scale    -> world_size

Each env's NEXT episode parameters are drawn ahead (torch RNG on the device) into
`env_cfg_next`; the step kernel switches an env to them when it resets it, and `after_step()`
draws fresh ones for exactly the envs the step reset (mask from env_done, no host sync).  The
entries without a counterpart in the swarm env — mass_scale (the kinematic env has no mass; the
physics restatement has no mass parameter), actuation delay / thrust noise and sensing noise
(they would change the observation contract the parity tests pin) — are reported in
`unsupported`, not silently dropped.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any

import torch

from . import _native as nat

SUPPORTED = {
    ("dynamics", "max_accel_scale"): "max_accel",
    ("dynamics", "max_speed_scale"): "max_speed",
    ("dynamics", "dt_scale"): "dt",
    ("environment", "obstacle_radius_scale"): "obstacle_radius",
    ("environment", "world_size_scale"): "world_size",
}


def load_dr_config(path: str | Path) -> dict[str, Any]:
    """The randomisation mapping from YAML (yaml.safe_load: data only) or JSON."""
    p = Path(path)
    text = p.read_text(encoding="utf-8")
    if p.suffix.lower() == ".json":
        import json
        cfg = json.loads(text)
    else:
        import yaml
        cfg = yaml.safe_load(text)
    if not isinstance(cfg, dict) or not isinstance(cfg.get("randomization"), dict):
        raise ValueError(f"no 'randomization' mapping in {p}")
    return cfg


def scale_ranges(dr_cfg: dict, profile: str = "train", physics: bool = False):
    """({param: (lo, hi)} of the supported uniform scale entries, [unsupported 'group.name']).
    profile 'ood' takes min/max from evaluation.out_of_distribution_profile where it names them."""
    if profile not in ("train", "ood"):
        raise ValueError(f"profile must be 'train' or 'ood', got {profile!r}")
    ood = ((dr_cfg.get("evaluation") or {}).get("out_of_distribution_profile") or {}) if profile == "ood" else {}
    ranges, unsupported = {}, []
    for group, entries in (dr_cfg.get("randomization") or {}).items():
        for name, spec in (entries or {}).items():
            param = SUPPORTED.get((group, name))
            spec = dict(spec or {})
            spec.update(ood.get(name) or {})
            if param is None or (physics and param == "dt") or spec.get("distribution", "uniform") != "uniform":
                unsupported.append(f"{group}.{name}")
                continue
            lo, hi = float(spec["min"]), float(spec["max"])
            if not (0.0 < lo <= hi):
                raise ValueError(f"{group}.{name}: need 0 < min <= max, got [{lo}, {hi}]")
            ranges[param] = (lo, hi)
    listed = {name for entries in (dr_cfg.get("randomization") or {}).values() for name in (entries or {})}
    unsupported += [f"evaluation.{name}" for name in ood if name not in listed]
    return ranges, unsupported


def sample_values(base: dict[str, float], ranges: dict, e: int, generator: torch.Generator,
                  device) -> dict[str, torch.Tensor]:
    """base[param] * U(lo, hi) per env, float64 [E] tensors on `device`."""
    out = {}
    for param in sorted(ranges):
        lo, hi = ranges[param]
        u = torch.rand((e,), generator=generator, dtype=torch.float64, device=device)
        out[param] = float(base[param]) * (lo + (hi - lo) * u)
    return out


class DomainRandomizer:
    """Per-episode parameter draws for a VecSwarm (see the module docstring)."""

    def __init__(self, vec, dr_cfg: dict | str | Path, *, seed: int = 0, profile: str = "train",
                 force: bool = False):
        cfg = dr_cfg if isinstance(dr_cfg, dict) else load_dr_config(dr_cfg)
        self.vec = vec
        self.enabled = bool(cfg.get("enabled", False)) or force
        self.ranges, self.unsupported = scale_ranges(cfg, profile, physics=vec.dynamics == "physics")
        self.base = {p: float(getattr(vec.cfg, p)) for p in set(SUPPORTED.values())}
        self.generator = torch.Generator(device=vec.device)
        self.generator.manual_seed(int(seed))
        self._mask = None

    def sample(self) -> dict[str, torch.Tensor]:
        return sample_values(self.base, self.ranges, self.vec.num_envs, self.generator, self.vec.device)

    def begin(self, reset: bool = True):
        """Start every env on its own draw and queue a different draw for its next episode.

        A device reset copies `env_cfg_next` into the current record (swarm_kernel.hip draw_env),
        so the first episode's draw goes into `next`, the reset switches it in, and a fresh draw
        then refills `next` — otherwise the first two episodes of every env would share one draw.
        reset=True performs that vec.reset() here and returns its obs; with reset=False the
        caller must reset and then call `after_reset()`."""
        if not self.enabled or not self.ranges:
            return self.vec.reset() if reset else None
        self.vec.set_env_config(**self.sample())  # current records exist before the first reset
        self.vec.set_env_config(next_episode=True, **self.sample())
        if not reset:
            return None
        obs = self.vec.reset()
        self.after_reset()
        return obs

    def after_reset(self, env_mask: torch.Tensor | None = None) -> None:
        """Fresh next-episode draws for the envs an explicit vec.reset(env_mask) just started
        (all if None): the reset consumed their queued draw."""
        if not self.enabled or not self.ranges:
            return
        self.vec.set_env_config(next_episode=True, env_mask=env_mask, **self.sample())

    def after_step(self) -> None:
        """Fresh next-episode draws for the envs the last step reset (they started the drawn
        ones).  Device-only: the mask comes from env_done on the device."""
        if not self.enabled or not self.ranges:
            return
        self.vec.join()
        self._mask = (self.vec.env_done & nat.ENV_RESET) != 0
        self.vec.set_env_config(next_episode=True, env_mask=self._mask, **self.sample())
