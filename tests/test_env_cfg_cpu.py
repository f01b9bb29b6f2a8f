"""CPU: per-env parameters — the per-env oracle, the domain-randomisation config mapping and the
mixed-stage curriculum validation (no GPU).

The per-env oracle (oracle/env_cfg_oracle.py) must reduce to the batch oracle when every env holds
the batch config (it is then the same computation env by env), and must equal a separate
single-env batch per distinct config when they differ.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

DR_YAML = """
version: 1
enabled: false
apply_on_reset: true
randomization:
  dynamics:
    mass_scale: {distribution: uniform, min: 0.85, max: 1.15}
    max_accel_scale: {distribution: uniform, min: 0.90, max: 1.10}
    max_speed_scale: {distribution: uniform, min: 0.90, max: 1.10}
    dt_scale: {distribution: uniform, min: 0.95, max: 1.05}
  actuation:
    control_delay_steps: {distribution: discrete, values: [0, 1, 2], probs: [0.7, 0.2, 0.1]}
    thrust_noise_std: {distribution: normal, mean: 0.0, std: 0.03}
  sensing:
    position_noise_std: {distribution: normal, mean: 0.0, std: 0.02}
  environment:
    obstacle_radius_scale: {distribution: uniform, min: 0.9, max: 1.1}
    world_size_scale: {distribution: uniform, min: 0.95, max: 1.05}
evaluation:
  use_randomization: true
  out_of_distribution_profile:
    mass_scale: {min: 0.80, max: 1.20}
    max_accel_scale: {min: 0.85, max: 1.15}
    control_delay_steps: {values: [0, 1, 2, 3], probs: [0.5, 0.25, 0.15, 0.10]}
"""


def _rollout_state(cfg, e, seed=3):
    from oracle import swarm_oracle as so
    st = so.empty_state(cfg, e)
    st, _ = so.reset_device(cfg, st, seed=seed)
    return st


def test_uniform_per_env_oracle_equals_batch_oracle():
    from oracle import env_cfg_oracle as eco
    from oracle import swarm_oracle as so
    cfg = so.make_cfg(num_drones=5, num_obstacles=6, max_steps=5)
    e = 6
    st = _rollout_state(cfg, e)
    st_b = {k: v.copy() for k, v in st.items()}
    rng = np.random.default_rng(0)
    for t in range(8):
        a = rng.uniform(-2, 2, (e, 5, 3)).astype(np.float32)
        st, out, _ = eco.step(cfg, {}, st, a, seed=3)
        st_b, out_b = so.step(cfg, st_b, a, auto_reset=True, seed=3)
        for k in ("obs", "reward", "terminated", "truncated", "term_all", "trunc_all", "reset", "global_state"):
            assert np.array_equal(out[k], out_b[k]), (t, k)
        for k in st:
            assert np.array_equal(st[k], st_b[k]), (t, k)


def test_per_env_oracle_equals_single_config_batches():
    """Envs with differing configs == separate batches of one config each (env_offset = index)."""
    from oracle import env_cfg_oracle as eco
    from oracle import swarm_oracle as so
    base = so.make_cfg(num_drones=4, num_obstacles=5)
    over = dict(world_size=np.array([14.0, 26.0, 20.0]), max_steps=np.array([4, 7, 5], np.int32),
                num_obstacles=np.array([0, 5, 2], np.int32), dt=np.array([0.1, 0.07, 0.15]))
    st = so.empty_state(base, 3)
    st, _ = eco.reset(base, over, st, seed=9)
    singles = []
    for e in range(3):
        c = eco.env_cfg(base, over, e)
        s1 = so.empty_state(c, 1)
        s1, _ = so.reset_device(c, s1, seed=9, env_offset=e)
        singles.append((c, s1))
        assert np.array_equal(st["pos"][e], s1["pos"][0])
        assert np.array_equal(st["obst"][e, :c["num_obstacles"]], s1["obst"][0])
        assert not st["obst"][e, c["num_obstacles"]:].any()
    rng = np.random.default_rng(1)
    for t in range(9):
        a = rng.uniform(-2, 2, (3, 4, 3)).astype(np.float32)
        st, out, _ = eco.step(base, over, st, a, seed=9)
        for e, (c, s1) in enumerate(singles):
            s1, o1 = so.step(c, s1, a[e:e + 1], auto_reset=True, seed=9, env_offset=e)
            singles[e] = (c, s1)
            assert np.array_equal(out["obs"][e], o1["obs"][0]), (t, e)
            assert np.array_equal(out["reward"][e], o1["reward"][0]), (t, e)


def test_dr_scale_ranges(tmp_path):
    import yaml
    from swarm_marl_amd.domain_randomization import load_dr_config, scale_ranges
    p = tmp_path / "dr.yaml"
    p.write_text(DR_YAML)
    cfg = load_dr_config(p)
    assert cfg == yaml.safe_load(DR_YAML)
    ranges, unsupported = scale_ranges(cfg)
    assert ranges == {"max_accel": (0.9, 1.1), "max_speed": (0.9, 1.1), "dt": (0.95, 1.05),
                      "obstacle_radius": (0.9, 1.1), "world_size": (0.95, 1.05)}
    assert set(unsupported) == {"dynamics.mass_scale", "actuation.control_delay_steps",
                                "actuation.thrust_noise_std", "sensing.position_noise_std"}
    ood, _ = scale_ranges(cfg, "ood")
    assert ood["max_accel"] == (0.85, 1.15) and ood["max_speed"] == (0.9, 1.1)
    phys, unsup_p = scale_ranges(cfg, physics=True)
    assert "dt" not in phys and "dynamics.dt_scale" in unsup_p
    with pytest.raises(ValueError):
        scale_ranges(cfg, "bogus")
    bad = dict(cfg, randomization={"dynamics": {"max_speed_scale": {"min": 1.2, "max": 1.1}}})
    with pytest.raises(ValueError):
        scale_ranges(bad)
    (tmp_path / "none.yaml").write_text("enabled: true\n")
    with pytest.raises(ValueError):
        load_dr_config(tmp_path / "none.yaml")


def test_dr_reference_config_parses():
    from pathlib import Path
    from swarm_marl_amd.domain_randomization import load_dr_config, scale_ranges
    ref = Path("/root/reference/configs/domain_randomization_v1.yaml")
    if not ref.exists():
        pytest.skip("reference configs not present (GPU box)")
    cfg = load_dr_config(ref)
    assert cfg["enabled"] is False and cfg["apply_on_reset"] is True
    ranges, _ = scale_ranges(cfg)
    assert set(ranges) == {"max_accel", "max_speed", "dt", "obstacle_radius", "world_size"}


def test_dr_sample_values_bounds_and_determinism():
    from swarm_marl_amd.domain_randomization import sample_values
    base = {"max_speed": 4.0, "world_size": 20.0}
    ranges = {"max_speed": (0.9, 1.1), "world_size": (0.95, 1.05)}
    g = torch.Generator().manual_seed(3)
    v = sample_values(base, ranges, 5000, g, "cpu")
    assert v["max_speed"].dtype == torch.float64 and v["max_speed"].shape == (5000,)
    assert float(v["max_speed"].min()) >= 3.6 and float(v["max_speed"].max()) <= 4.4
    assert float(v["world_size"].min()) >= 19.0 and float(v["world_size"].max()) <= 21.0
    assert abs(float(v["max_speed"].mean()) - 4.0) < 0.02
    g2 = torch.Generator().manual_seed(3)
    assert torch.equal(sample_values(base, ranges, 5000, g2, "cpu")["max_speed"], v["max_speed"])


def test_mixed_stage_batch_validation():
    from swarm_marl_amd.curriculum import mixed_stage_batch
    cfg = {"stages": [{"env_config": {"num_drones": 3, "num_obstacles": 0}},
                      {"env_config": {"num_drones": 5, "num_obstacles": 4}},
                      {"env_config": {"num_drones": 3, "num_obstacles": 4, "neighbor_k": 2}}]}
    with pytest.raises(ValueError, match="num_drones"):
        mixed_stage_batch(cfg, [0, 1])
    with pytest.raises(ValueError, match="other than"):
        mixed_stage_batch(cfg, [0, 2])
    with pytest.raises(ValueError, match="out of range"):
        mixed_stage_batch(cfg, [0, 3])
    with pytest.raises(ValueError):
        mixed_stage_batch(cfg, [])
