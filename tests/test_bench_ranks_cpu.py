"""CPU, world_size 2 over gloo: bench.py's multi-rank logic with CPU stand-in steps.

The same functions bench.main() uses on the GPU (shard_plan, timed_region, max_over_ranks,
gather_schedule + the CTDE distributed.GlobalStateGather over a global_state slot ring) drive a C-oracle stand-in for the step on
each rank.  Checks: the weak-scaling shards equal one run over the whole batch (the reset RNG is
keyed by the global env index), every rank sees the MAX of the per-rank timings, and the
periodic global_state gather concatenates the shards in rank order at the scheduled steps.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N, E_PER, STEPS, EVERY = 5, 6, 7, 3


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _actions(world: int, t: int) -> np.ndarray:
    return np.random.default_rng(500 + t).uniform(-1, 1, (world * E_PER, N, 3)).astype(np.float32)


def _worker(rank: int, world: int, port: int, outdir: str) -> None:
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle import c_oracle as co
        from oracle import swarm_oracle as so
        off, cnt = bench.shard_plan(world, rank, E_PER)
        cfg = so.make_cfg(num_drones=N, max_steps=4)
        run = co.Runner(cfg, cnt, seed=9, env_offset=off, nthreads=1)
        from swarm_marl_amd.distributed import GlobalStateGather
        sched = set(bench.gather_schedule(STEPS, EVERY))
        # bench.main's CTDE gather: a 3-slot global_state ring, slot k % 3 written by step k
        ring = torch.full((3, cnt, 6 * N + 3), float("nan"))
        slot = {}
        g = GlobalStateGather(ring, lambda i: slot.__setitem__("cur", i), keep=8)
        gathered, obs = {}, []

        def body():
            for k in range(STEPS):
                s = g.before_step()
                assert s == slot["cur"] == k % 3
                run.step(_actions(world, k)[off:off + cnt])
                ring[s].copy_(torch.from_numpy(run.out["global_state"]))  # the kernel's write-back
                obs.append(run.out["obs"].copy())
                g.after_step(gather=k in sched)
                if k in sched:
                    g.wait()
                    gathered[k] = g.result().numpy().copy()
            assert g.gathered_steps == sorted(sched)
        wall = bench.timed_region(body, world, lambda: None)
        # rank-dependent stand-in timings: every rank must get the max
        m = bench.max_over_ranks([wall, 1.0 + rank, 10.0 - rank], world)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), obs=np.stack(obs), off=off, cnt=cnt,
                 m=np.array(m), gk=np.array(sorted(gathered)),
                 g=np.stack([gathered[k] for k in sorted(gathered)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bench_rank_logic_gloo(tmp_path):
    import bench
    from oracle import c_oracle as co
    from oracle import swarm_oracle as so
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    cfg = so.make_cfg(num_drones=N, max_steps=4)
    run = co.Runner(cfg, world * E_PER, seed=9, nthreads=1)
    ref_obs, ref_gs = [], {}
    sched = bench.gather_schedule(STEPS, EVERY)
    for k in range(STEPS):
        run.step(_actions(world, k))
        ref_obs.append(run.out["obs"].copy())
        if k in sched:
            ref_gs[k] = run.out["global_state"].copy()
    ref_obs = np.stack(ref_obs)
    assert np.any(run.st["episode"] > 0), "the run should cross episode boundaries"
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        off, cnt = int(d["off"]), int(d["cnt"])
        assert (off, cnt) == (r * E_PER, E_PER)
        assert np.array_equal(d["obs"], ref_obs[:, off:off + cnt]), f"rank {r} obs"
        assert d["m"][1] == 1.0 + (world - 1) and d["m"][2] == 10.0, "max over ranks"
        assert d["gk"].tolist() == sched
        for i, k in enumerate(sched):
            assert np.array_equal(d["g"][i], ref_gs[k]), f"rank {r} gathered global_state @ {k}"


def test_gather_schedule_and_shards():
    import bench
    assert bench.gather_schedule(7, 3) == [2, 5, 6]
    assert bench.gather_schedule(6, 3) == [2, 5]
    assert bench.gather_schedule(5, 8) == [4]
    assert bench.shard_plan(8, 3, 8192) == (3 * 8192, 8192)
    with pytest.raises(ValueError):
        bench.shard_plan(2, 2, 10)


def test_bench_args_presets():
    import bench
    a = bench.parse([])
    assert (a.drones, a.envs, a.ctde) == (64, 8192, False)
    a = bench.parse(["--config", "n16"])
    assert (a.drones, a.envs, a.ctde) == (16, 1024, False)
    a = bench.parse(["--config", "n256"])
    assert (a.drones, a.envs, a.ctde) == (256, 1024, True)
    a = bench.parse(["--config", "n256", "--envs", "64"])
    assert a.envs == 64


def _run_bench(args, env_extra, timeout=240):
    import subprocess
    import sys
    from pathlib import Path
    ROOT = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=env, cwd=str(ROOT),
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(300)
def test_plain_bench_gpus2_spawns_two_ranks():
    """`python bench.py --gpus 2` (no torchrun) launches 2 ranks itself (CPU stand-in step)."""
    import json
    p = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--envs", "16"],
                   {"SWARM_BENCH_STANDIN": "cpu"})
    assert p.returncode == 0, p.stderr[-2000:]
    rec = [json.loads(s) for s in p.stdout.splitlines() if s.startswith("{")]
    assert len(rec) == 1, p.stdout
    r = rec[0]
    assert r["n_gpus"] == 2 and r["world_size"] == 2
    assert [d["rank"] for d in r["rank_devices"]] == [0, 1]
    assert [d["env_offset"] for d in r["rank_devices"]] == [0, 16]
    assert r["config"]["global_envs"] == 32


@pytest.mark.timeout(120)
def test_bench_gpus_more_than_visible_fails():
    """--gpus 8 with fewer visible GPUs (none here) fails loudly before any rank starts."""
    p = _run_bench(["--gpus", "8", "--steps", "2"], {})
    assert p.returncode != 0
    assert "needs 8 GPUs" in p.stderr


def test_check_world_rules():
    import bench
    assert bench.check_world(1, env={}, device_count=1) == (1, None)
    assert bench.check_world(4, env={}, device_count=8) == (4, "launch")
    assert bench.check_world(2, env={"WORLD_SIZE": "2"}, device_count=2) == (2, None)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 4"):
        bench.check_world(4, env={"WORLD_SIZE": "2"}, device_count=8)
    with pytest.raises(SystemExit, match="needs 8 GPUs"):
        bench.check_world(8, env={}, device_count=1)
    # the one-GPU rehearsal shares cuda:0
    assert bench.check_world(2, env={"SWARM_BENCH_REHEARSAL": "1"}, device_count=1) == (2, "launch")


@pytest.mark.timeout(300)
def test_launcher_fails_when_a_rank_fails():
    """A rank that fails makes the launcher exit non-zero (rank 1 gets a bad env count)."""
    p = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--envs", "-1"],
                   {"SWARM_BENCH_STANDIN": "cpu"})
    assert p.returncode != 0
