"""GPU: BASELINE.json configs 4 and 5 exercised at their per-GPU workload on one MI355X.

config 4  N=64 x E=65536 envs sharded env-parallel over 8 GPUs (no collectives): the whole
          65536-env batch stepped in one launch must equal the 8 rank shards of 8192 envs
          (env_offset = r * 8192) bit for bit — obs, reward, flags, state — over 6 steps with
          in-kernel resets; the persistent env-queue kernel must equal the one-shot launch; and a
          64-env slice must match the CPU oracle (bit-exact obs, rewards within 1e-5).
config 5  N=256 x E=8192 over 8 GPUs with the CTDE global_state all-gather: one rank's slab,
          N=256 x E=1024 with global_state, 4 auto-reset steps; a 16-env slice against the oracle
          and the whole slab against the observation / global_state invariants.
Reference: src/swarm_marl/envs/drone_swarm_env.py:92-174 (step), :226-291 (obs), :293-302
(global state).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from tests.helpers import oracle_cfg, vec_state_numpy

pytestmark = pytest.mark.gpu
REWARD_TOL = 1e-5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _actions(dev, t, e_total, n):
    g = torch.Generator(device=dev).manual_seed(7000 + t)
    return torch.rand((e_total, n, 3), device=dev, generator=g) * 2 - 1


def _snap(vec):
    return [t.clone() for t in (vec.obs, vec.reward, vec.terminated, vec.truncated, vec.env_done,
                                vec.pos, vec.vel, vec.goal, vec.obstacles, vec.active,
                                vec.step_count, vec.episode)]


def test_config4_full_batch_equals_rank_shards(dev):
    from swarm_marl_amd import VecSwarm
    e_all, e_rank, n, steps = 65536, 8192, 64, 6
    full = VecSwarm(e_all, {"num_drones": n}, device=dev, auto_reset=True, seed=3)
    full.reset()
    shards = [VecSwarm(e_rank, {"num_drones": n}, device=dev, auto_reset=True, seed=3,
                       env_offset=r * e_rank) for r in range(8)]
    for s in shards:
        s.reset()
    resets = 0
    for t in range(steps):
        a = _actions(dev, t, e_all, n)
        full.step(a)
        fs = _snap(full)
        for r, s in enumerate(shards):
            s.step(a[r * e_rank:(r + 1) * e_rank].contiguous())
            for k, x in enumerate(_snap(s)):
                assert torch.equal(fs[k][r * e_rank:(r + 1) * e_rank], x), f"t={t} rank={r} field {k}"
        resets += int(((fs[4] & 4) != 0).sum())
    assert resets > 1000, "the run must cross many episode boundaries"


def test_config4_persistent_grid_equals_one_shot(dev):
    from swarm_marl_amd import VecSwarm
    e, n = 65536, 64
    a_vec = VecSwarm(e, {"num_drones": n}, device=dev, auto_reset=True, seed=5)
    b_vec = VecSwarm(e, {"num_drones": n}, device=dev, auto_reset=True, seed=5, waves_per_simd=4)
    assert b_vec.kernel_name() == "swarm_step64<32>" and a_vec.kernel_name() != b_vec.kernel_name()
    a_vec.reset()
    b_vec.reset()
    for t in range(4):
        a = _actions(dev, t, e, n)
        a_vec.step(a)
        b_vec.step(a)
        for x, y in zip(_snap(a_vec), _snap(b_vec)):
            assert torch.equal(x, y), f"t={t}"
    assert int(b_vec.work.abs().sum()) == 0, "queue heads must be left at zero"


def test_config4_slice_vs_oracle(dev):
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    e, n = 65536, 64
    vec = VecSwarm(e, {"num_drones": n}, device=dev, auto_reset=True, seed=11, with_infos=True,
                   with_global_state=True)
    vec.reset()
    cfg = oracle_cfg({"num_drones": n})
    lo = e - 64  # the last 64 envs: the highest global env indices of the launch
    for t in range(3):
        pre = vec_state_numpy(vec)
        a = _actions(dev, t, e, n)
        vec.step(a)
        st = {k: v[lo:] for k, v in pre.items()}
        ns, out = so.step(cfg, st, a[lo:].cpu().numpy(), auto_reset=True, seed=11, env_offset=lo)
        assert np.array_equal(vec.obs[lo:].cpu().numpy(), out["obs"]), f"obs t={t}"
        err = np.abs(vec.reward[lo:].cpu().numpy().astype(np.float64) - out["reward"]).max()
        assert err <= REWARD_TOL, f"reward t={t}: {err}"
        assert np.array_equal(vec.pos[lo:].cpu().numpy(), ns["pos"])
        assert np.array_equal(vec.global_state[lo:].cpu().numpy(), out["global_state"])


def test_config5_slab_n256_global_state(dev):
    from oracle import swarm_oracle as so
    from swarm_marl_amd import VecSwarm
    e, n = 1024, 256
    vec = VecSwarm(e, {"num_drones": n}, device=dev, auto_reset=True, seed=2, with_infos=True,
                   with_global_state=True)
    vec.reset()
    cfg = oracle_cfg({"num_drones": n})
    sl = slice(100, 116)  # a 16-env slice
    resets = 0
    for t in range(4):
        pre = vec_state_numpy(vec)
        a = _actions(dev, t, e, n)
        vec.step(a)
        torch.cuda.synchronize()
        st = {k: v[sl] for k, v in pre.items()}
        ns, out = so.step(cfg, st, a[sl].cpu().numpy(), auto_reset=True, seed=2, env_offset=100)
        assert np.array_equal(vec.obs[sl].cpu().numpy(), out["obs"]), f"obs t={t}"
        err = np.abs(vec.reward[sl].cpu().numpy().astype(np.float64) - out["reward"]).max()
        assert err <= REWARD_TOL, f"reward t={t}: {err}"
        assert np.array_equal(vec.global_state[sl].cpu().numpy(), out["global_state"])
        env_done = (out["term_all"].astype(np.uint8) | (out["trunc_all"].astype(np.uint8) << 1)
                    | (out["reset"].astype(np.uint8) << 2))
        assert np.array_equal(vec.env_done[sl].cpu().numpy(), env_done)
        # whole slab: observation / global_state invariants of the post-step state
        obs, pos, vel, goal, gs = vec.obs, vec.pos, vec.vel, vec.goal, vec.global_state
        assert torch.equal(obs[..., 0:3], pos) and torch.equal(obs[..., 3:6], vel)
        assert torch.equal(obs[..., 6:9], goal[:, None, :] - pos)
        nd = obs[..., 9:21].reshape(e, n, 3, 4)[..., 3]
        od = obs[..., 21:37].reshape(e, n, 4, 4)[..., 3]
        assert bool((nd[..., 1:] >= nd[..., :-1]).all()) and bool((nd > 0).all())
        assert bool((od[..., 1:] >= od[..., :-1]).all())
        assert torch.equal(gs[:, :3 * n].reshape(e, n, 3), pos)
        assert torch.equal(gs[:, 3 * n:6 * n].reshape(e, n, 3), vel)
        assert torch.equal(gs[:, 6 * n:], goal)
        resets += int(((vec.env_done & 4) != 0).sum())
    assert resets > 0
