"""Shared test helpers (fixture loading, state conversion)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"

ROLLOUT_FIXTURES = sorted(p.name for p in GOLDEN.glob("*.npz")
                          if not p.name.startswith(("reset_", "single", "policy_", "eval")))


def load_fixture(name: str):
    d = np.load(GOLDEN / name)
    cfg = json.loads(str(d["config"]))
    return d, cfg


def oracle_cfg(raw: dict):
    from oracle import swarm_oracle as so
    return so.make_cfg(**raw)


def vec_state_numpy(vec) -> dict:
    """VecSwarm state tensors -> oracle-convention numpy dict."""
    s = {k: v.detach().cpu().numpy() for k, v in vec.state_dict().items()}
    return dict(pos=s["pos"], vel=s["vel"], goal=s["goal"], obst=s["obstacles"],
                active=s["active"].astype(bool), step=s["step_count"],
                episode=s["episode"].view(np.uint32), damping=s["damping"])
