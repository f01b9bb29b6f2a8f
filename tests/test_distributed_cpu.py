"""CPU, world_size 2 over gloo: the env-sharded multi-GPU path, rehearsed on host processes.

Each rank owns a contiguous env shard (distributed.shard_bounds) and steps it with no collective;
the in-kernel reset RNG is keyed by the GLOBAL env index (env_offset), so the shards together
must equal a single run over the whole batch.  The only exchange, the CTDE global_state
all-gather (distributed.gather_global_state), must concatenate the shards in rank order.
The per-rank stepping uses the C oracle (same state conventions and env_offset semantics as the
kernel's C-ABI), so this runs without a GPU.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

E_GLOBAL, N, STEPS, SEED = 10, 6, 7, 21


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _actions(t: int) -> np.ndarray:
    return np.random.default_rng(1000 + t).uniform(-1, 1, (E_GLOBAL, N, 3)).astype(np.float32)


def _worker(rank: int, world: int, port: int, outdir: str) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import c_oracle as co
        from oracle import swarm_oracle as so
        from swarm_marl_amd.distributed import gather_global_state, shard_bounds
        off, cnt = shard_bounds(E_GLOBAL, world, rank)
        cfg = so.make_cfg(num_drones=N, max_steps=3)  # short episodes: several in-step resets
        st, out = co.run(cfg, so.empty_state(cfg, cnt), "reset", seed=SEED, env_offset=off)
        obs_all, gs_all = [out["obs"]], []
        for t in range(STEPS):
            a = _actions(t)[off:off + cnt]
            st, out = co.run(cfg, st, "step", a, auto_reset=True, seed=SEED, env_offset=off)
            obs_all.append(out["obs"])
            # weak-scaling shards are equal-sized here (10 / 2)
            g = gather_global_state(torch.from_numpy(out["global_state"]))
            gs_all.append(g.numpy())
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), obs=np.stack(obs_all),
                 gs=np.stack(gs_all), off=off, cnt=cnt)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_run_equals_single_run(tmp_path):
    from oracle import c_oracle as co
    from oracle import swarm_oracle as so
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    cfg = so.make_cfg(num_drones=N, max_steps=3)
    st, out = co.run(cfg, so.empty_state(cfg, E_GLOBAL), "reset", seed=SEED)
    ref_obs, ref_gs = [out["obs"]], []
    for t in range(STEPS):
        st, out = co.run(cfg, st, "step", _actions(t), auto_reset=True, seed=SEED)
        ref_obs.append(out["obs"])
        ref_gs.append(out["global_state"])
    ref_obs, ref_gs = np.stack(ref_obs), np.stack(ref_gs)
    assert np.any(st["episode"] > 0), "the run should cross episode boundaries"
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        off, cnt = int(d["off"]), int(d["cnt"])
        assert np.array_equal(d["obs"], ref_obs[:, off:off + cnt]), f"rank {r} obs"
        assert np.array_equal(d["gs"], ref_gs), f"rank {r} gathered global_state"
