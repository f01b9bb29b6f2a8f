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


def test_rank_process_group_and_groups(monkeypatch):
    """A rank holds an RCCL communicator only for the CTDE gather (r06l / r06m: one in the process
    slowed the driver's command by 10-15 %), and only a gathering rank drops to 2 env groups."""
    import bench
    assert bench.pg_backend(ctde=False, rehearsal=False) == "gloo"
    assert bench.pg_backend(ctde=True, rehearsal=False) == "nccl"
    assert bench.pg_backend(ctde=True, rehearsal=True) == "gloo"
    monkeypatch.setenv("WORLD_SIZE", "4")
    args = ["--gpus", "4", "--steps", "20", "--warmup", "5"]
    assert bench.parse(args).groups == bench.PRESETS["headline"]["groups"]
    assert bench.parse(args + ["--config", "n256"]).groups == min(bench.PRESETS["n256"]["groups"], 2)
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.parse(args[:0] + ["--steps", "20", "--config", "n256"]).groups == bench.PRESETS["n256"]["groups"]


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
    """Only rank 1 fails; rank 0 is then blocked in the timed region's barrier and must be stopped
    by the launcher, which exits non-zero well inside the timeout (gloo's own barrier timeout is
    30 minutes)."""
    import time
    t0 = time.perf_counter()
    p = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--envs", "4"],
                   {"SWARM_BENCH_STANDIN": "cpu", "SWARM_BENCH_STANDIN_FAIL_RANK": "1"}, timeout=200)
    assert p.returncode != 0
    assert "rank 1 exited" in p.stderr, p.stderr[-2000:]
    assert not [s for s in p.stdout.splitlines() if s.startswith("{")]  # rank 0 never reported
    assert time.perf_counter() - t0 < 150


_PARENT_PROBE = r"""
import json, subprocess, sys
sys.argv = ["bench.py", *sys.argv[1:]]
import bench
real = subprocess.Popen
seen = []
class Spy(real):
    def __init__(self, cmd, *a, **k):
        # the parent's state at every child it starts: the device-count child and each rank
        maps = open("/proc/self/maps").read()
        torch_in = "torch" in sys.modules
        cuda_init = bool(torch_in and sys.modules["torch"].cuda.is_initialized())
        seen.append({"cmd": " ".join(map(str, cmd))[-60:], "torch_imported": torch_in,
                     "cuda_initialized": cuda_init, "hip_mapped": "libamdhip64" in maps})
        super().__init__(cmd, *a, **k)
subprocess.Popen = Spy
msg = ""
try:
    rc = bench.entry()
except SystemExit as e:
    rc = 1 if e.code is None or isinstance(e.code, str) else e.code
    msg = str(e.code)
print("PROBE " + json.dumps({"rc": rc, "msg": msg, "seen": seen}), file=sys.stderr)
sys.exit(0)
"""


def _probe(args, env_extra):
    import json
    import subprocess
    import sys
    from pathlib import Path
    ROOT = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra, PYTHONPATH=str(ROOT))
    p = subprocess.run([sys.executable, "-c", _PARENT_PROBE, *args], env=env, cwd=str(ROOT),
                       capture_output=True, text=True, timeout=240)
    line = [s for s in p.stderr.splitlines() if s.startswith("PROBE ")]
    assert line, p.stderr[-2000:]
    return json.loads(line[-1][6:]), p


@pytest.mark.timeout(300)
def test_launcher_parent_never_initialises_hip():
    """The launcher branch of `python bench.py --gpus N`: at every child it starts (the device-count
    child, then the ranks) the parent has not imported torch, so torch.cuda is not initialised and
    libamdhip64 is not mapped (exec-after-HIP-init is forbidden on the GPU pool, and a parent holding
    a HIP context would share the card with its ranks)."""
    # no GPU here: the device-count child reports 0 and the launch stops before any rank starts
    r, p = _probe(["--gpus", "2", "--steps", "2"], {})
    assert r["rc"] != 0 and "needs 2 GPUs" in r["msg"]
    assert len(r["seen"]) == 1 and "device_count" in r["seen"][0]["cmd"]
    # the CPU stand-in skips the count: the parent starts both ranks, still HIP-free
    r, p = _probe(["--gpus", "2", "--steps", "2", "--warmup", "1", "--envs", "4"], {"SWARM_BENCH_STANDIN": "cpu"})
    assert r["rc"] == 0, p.stderr[-2000:]
    assert len(r["seen"]) == 2
    for s in r["seen"]:
        assert not s["torch_imported"] and not s["cuda_initialized"] and not s["hip_mapped"], s


@pytest.mark.timeout(300)
def test_standin_ctde_gpus2_gathers():
    """`bench.py --config n256 --ctde --gpus 2` on the CPU stand-in: main()'s CTDE branch — the
    global_state slot ring all-gathered over gloo every --gather-every steps inside the timed
    region, shards concatenated in rank order."""
    import json
    p = _run_bench(["--config", "n256", "--ctde", "--gpus", "2", "--steps", "10", "--warmup", "1",
                    "--envs", "4", "--gather-every", "4"], {"SWARM_BENCH_STANDIN": "cpu"})
    assert p.returncode == 0, p.stderr[-2000:]
    rec = [json.loads(s) for s in p.stdout.splitlines() if s.startswith("{")]
    assert len(rec) == 1
    c = rec[0]["config"]
    assert c["ctde_allgather"] is True and c["ctde_gather_backend"] == "gloo"
    assert c["ctde_gathers_timed"] == len([3, 7, 9]) and c["ctde_rank_order_ok"] is True
    assert rec[0]["world_size"] == 2 and c["global_envs"] == 8


def test_valu_roofline_from_committed_pmc():
    """bench.valu_roofline: the committed PMC record of the headline gives the 2-cycle lower bound,
    the class-costed busy bracket and the SQ_ACTIVE_INST_VALU figure; the line's bound becomes
    "valu" when the class-costed busy fraction exceeds the HBM fraction (round-5 review ask)."""
    import json
    from pathlib import Path
    import bench
    prof = json.loads((Path(bench.ROOT) / "profiles" / "pmc_traffic.json").read_text())["kinematic+swarm N=64 E=8192"]
    v = bench.valu_roofline(prof, 0.0227)
    lo, hi = v["busy_class_costed"]
    assert v["frac_2cycle"] < lo <= hi == v["busy_frac"]
    assert 0.3 < hi < 1.2 and 0.3 < v["counter_frac"] < 1.2
    assert "lower bound" in v["frac_2cycle_note"]
    # per-SIMD issue time: waves per SIMD x ns per wave
    assert abs(v["valu_issue_us_per_simd_per_step"][1] - prof["valu_issue_ns_per_wave"][1] * 8e-3) < 1e-2
