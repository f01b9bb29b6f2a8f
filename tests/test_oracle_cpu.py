"""CPU: the oracles (numpy restatement + C port) pinned to the reference's golden fixtures.

The fixtures (tests/golden/*.npz, generated from the reference by tests/golden/make_golden.py)
hold the reference's own outputs step by step.  Both oracles must reproduce them bit-exactly:
observations, state, flags and the float64 rewards.  The C oracle must also agree with the numpy
oracle on random batched multi-step runs (auto-reset, physics, masked actions).
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import ROLLOUT_FIXTURES, load_fixture, oracle_cfg


def _fixture_state(d):
    e = d["pre_pos"].shape[0]
    return dict(pos=d["pre_pos"], vel=d["pre_vel"], goal=d["pre_goal"], obst=d["pre_obst"],
                active=d["pre_active"], step=d["pre_step"].astype(np.int32),
                episode=np.zeros(e, np.uint32), damping=np.zeros(d["pre_pos"].shape[:2], np.float32))


def _check_against_fixture(d, st, out, rew_exact=True):
    op = d["obs_present"]
    assert np.array_equal(out["obs"][op], d["out_obs"][op]), "obs"
    rp = d["rew_present"]
    if rp.any():
        if rew_exact:
            assert np.array_equal(out["reward"][rp], d["rew"][rp]), "reward (bit-exact)"
        else:
            assert np.abs(out["reward"][rp] - d["rew"][rp]).max() <= 1e-12
    tp = d["term_present"]
    assert np.array_equal(out["terminated"][tp].astype(bool), d["term"][tp])
    assert np.array_equal(out["truncated"][tp].astype(bool), d["trunc"][tp])
    assert np.array_equal(st["pos"], d["post_pos"])
    assert np.array_equal(st["vel"], d["post_vel"])
    assert np.array_equal(np.asarray(st["active"]).astype(bool), d["post_active"])
    assert np.array_equal(st["step"], d["post_step"])
    assert np.array_equal(out["global_state"], d["global_state"])
    ip = d["info_present"]
    assert np.array_equal(out["dist_goal"][ip].astype(np.float64), d["info_dist"][ip])


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_numpy_oracle_matches_reference_fixture(name):
    from oracle import swarm_oracle as so
    d, raw = load_fixture(name)
    cfg = oracle_cfg(raw)
    st, out = so.step(cfg, _fixture_state(d), d["actions"], d["action_present"],
                      exact_formation=True)
    assert np.array_equal(out["term_all"], d["term_all"])
    assert np.array_equal(out["trunc_all"], d["trunc_all"])
    assert np.array_equal(out["reached"][d["info_present"]], d["info_reached"][d["info_present"]])
    assert np.array_equal(out["collision"][d["info_present"]],
                          d["info_collision"][d["info_present"]])
    _check_against_fixture(d, st, out)


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_c_oracle_matches_reference_fixture(name):
    from oracle import c_oracle as co
    d, raw = load_fixture(name)
    cfg = oracle_cfg(raw)
    st, out = co.run(cfg, _fixture_state(d), "step", d["actions"], d["action_present"])
    ed = out["env_done"]
    assert np.array_equal((ed & 1) != 0, d["term_all"])
    assert np.array_equal((ed & 2) != 0, d["trunc_all"])
    _check_against_fixture(d, st, out)


@pytest.mark.parametrize("n,e,physics,k,ms,m", [
    (4, 40, False, 3, 4, 8), (16, 24, False, 3, 4, 8), (64, 6, False, 3, 4, 8),
    (33, 5, False, 5, 6, 7), (1, 30, False, 3, 4, 8), (24, 8, False, 0, 0, 0),
    (4, 20, True, 3, 4, 8), (16, 6, True, 3, 4, 8),
])
def test_c_oracle_matches_numpy_oracle_multistep(n, e, physics, k, ms, m):
    from oracle import c_oracle as co
    from oracle import swarm_oracle as so
    cfg = so.make_cfg(num_drones=n, neighbor_k=k, sensed_obstacles=ms, num_obstacles=m,
                      max_steps=4)
    st_n, _ = so.reset_device(cfg, so.empty_state(cfg, e), physics=physics, seed=5, env_offset=3)
    st_c, out_c = co.run(cfg, so.empty_state(cfg, e), "reset", physics=physics, seed=5,
                         env_offset=3)
    for key in ("pos", "goal", "obst", "damping"):
        assert np.array_equal(st_c[key], st_n[key]), key
    rng = np.random.default_rng(n + 100 * e)
    for t in range(6):
        a = rng.uniform(-1.2, 1.2, (e, n, 3)).astype(np.float32)
        am = rng.uniform(size=(e, n)) > 0.1
        st_n, out_n = so.step(cfg, st_n, a, am, physics=physics, auto_reset=True, seed=5,
                              env_offset=3, exact_formation=True)
        st_c, out_c = co.run(cfg, st_c, "step", a, am, physics=physics, auto_reset=True, seed=5,
                             env_offset=3)
        assert np.array_equal(out_c["obs"], out_n["obs"]), f"obs t={t}"
        assert np.array_equal(out_c["reward"], out_n["reward"]), f"reward t={t}"
        for key in ("pos", "vel", "goal", "obst", "step", "episode", "damping"):
            assert np.array_equal(st_c[key], st_n[key]), f"{key} t={t}"
        assert np.array_equal(st_c["active"].astype(bool), st_n["active"].astype(bool))
        assert np.array_equal((out_c["env_done"] & 4) != 0, out_n["reset"])


# Random123 known-answer vectors for philox4x32_10 (kat_vectors in the Random123 distribution)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(ctr, key, want):
    from oracle import c_oracle as co
    from oracle import swarm_oracle as so
    got = [int(x) for x in so.philox4x32_10(*ctr, *key)]
    assert got == list(want)
    assert co.philox4x32_10(ctr, key) == list(want)


def test_device_reset_draws_are_keyed_by_global_env():
    """Sharding invariance of the in-kernel reset stream: env g draws the same episode whatever
    shard it lives in, and different episodes / seeds draw differently."""
    from oracle import swarm_oracle as so
    cfg = so.make_cfg(num_drones=8)
    ids = np.arange(10, 30)
    ep = np.full(ids.shape, 3, np.uint32)
    full = so.device_reset_draws(cfg, ids, ep, seed=9)
    part = so.device_reset_draws(cfg, ids[7:], ep[7:], seed=9)
    for a, b in zip(full, part):
        assert np.array_equal(a[7:], b)
    other_ep = so.device_reset_draws(cfg, ids, ep + 1, seed=9)
    other_seed = so.device_reset_draws(cfg, ids, ep, seed=10)
    assert not np.array_equal(full[0], other_ep[0])
    assert not np.array_equal(full[0], other_seed[0])
    half = cfg["world_size"] / 2
    for arr in full[:3]:
        assert np.all(arr >= -half) and np.all(arr < half)
