#!/usr/bin/env python3
"""Headline benchmark: agent-steps/s of the fused swarm step at N=64 drones x E=8192 envs/GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one launch of the fused kernel over the local env shard (integrate, distances,
collision, formation, rewards, terminations, in-kernel auto-reset, kNN obs) with inputs resident
in HBM.  Envs are sharded across ranks with no collective on the step path (weak scaling:
8192 envs per GPU).  The K timed steps run twice: eagerly with HIP events around every launch
(per-launch kernel time for the roofline) and as hipGraph replays of the action-ring segment
(`value`: the whole-job rate without per-step host launch cost; --no-graph times the eager
loop instead).  Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic HBM bytes
per launch / mean kernel duration from HIP events on the launch stream;
`cpu_baseline` = the C oracle (oracle/swarm_oracle.c, a port of the reference step) timed on the
host cores for a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
sys.path.insert(0, str(ROOT))

METRIC = "agent-steps/sec at N=64 × E=8192 envs, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--drones", type=int, default=64)
    ap.add_argument("--envs", type=int, default=8192, help="envs per GPU")
    ap.add_argument("--no-term", action="store_true",
                    help="no-termination variant (collision/goal radii 0)")
    ap.add_argument("--ring", type=int, default=8, help="distinct pre-generated action tensors")
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--waves-per-simd", type=int, default=0,
                    help="persistent step kernel: resident waves per SIMD (0 = library default)")
    ap.add_argument("--no-persistent", action="store_true",
                    help="one workgroup per env instead of the persistent env queue")
    ap.add_argument("--no-graph", action="store_true",
                    help="time the whole-job rate with eager launches instead of hipGraph replay")
    ap.add_argument("--ctde", action="store_true",
                    help="also emit global_state and all-gather it every step (config 5)")
    return ap.parse_args()


def cpu_baseline(cfg_raw: dict, n: int, seconds: float) -> dict:
    """C oracle on the host cores: bounded sample of the same workload (auto-reset on)."""
    from oracle import c_oracle as co
    from oracle import swarm_oracle as so

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", "16")), 16))
    cfg = so.make_cfg(**cfg_raw)
    e = 64 * threads
    st = so.empty_state(cfg, e)
    st, _ = co.run(cfg, st, "reset", seed=0, nthreads=threads)
    rng = np.random.default_rng(1000)
    ring = [rng.uniform(-1, 1, (e, n, 3)).astype(np.float32) for _ in range(4)]
    co.run(cfg, st, "step", ring[0], auto_reset=True, nthreads=threads)  # warm
    steps, t0 = 0, time.perf_counter()
    while True:
        st, _ = co.run(cfg, st, "step", ring[steps % 4], auto_reset=True, seed=0,
                       nthreads=threads)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": e * n * steps / el, "unit": "agent-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"C oracle (port of DroneSwarmEnv.step, oracle/swarm_oracle.c), OpenMP "
                      f"{threads} threads, N={n} x E={e} envs, {steps} steps in {el:.2f} s, "
                      f"auto-reset on; includes ctypes call overhead per step"}


def pmc_traffic(workload_key: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary, if one matches."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
    except Exception:
        return None
    rec = d.get(workload_key)
    return None if rec is None else rec.get("hbm_bytes_per_launch")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from swarm_marl_amd import VecSwarm

    n, e = args.drones, args.envs
    raw = {"num_drones": n}
    if args.no_term:
        raw.update(collision_radius=0.0, obstacle_radius=0.0, goal_radius=0.0)
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=0, env_offset=rank * e,
                   with_global_state=args.ctde, persistent=not args.no_persistent,
                   waves_per_simd=args.waves_per_simd)
    vec.reset()
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    ring = [torch.rand((e, n, 3), device=dev, generator=gen) * 2 - 1 for _ in range(args.ring)]
    gather_buf = None
    if args.ctde and world > 1:
        gather_buf = torch.empty((world * e, 6 * n + 3), device=dev)

    def one(k):
        vec.step(ring[k % args.ring])
        if gather_buf is not None:
            dist.all_gather_into_tensor(gather_buf, vec.global_state)

    for k in range(args.warmup):
        one(k)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        vec.step(ring[k % args.ring])
        ev[k][1].record(stream)
        if gather_buf is not None:
            dist.all_gather_into_tensor(gather_buf, vec.global_state)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall_eager = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # Whole-job rate: the same K steps replayed from a hipGraph that holds one step launch per
    # action tensor of the ring (host launch cost off the step path, as in a captured rollout).
    wall, timing = wall_eager, "eager launches"
    if not args.no_graph and gather_buf is None:
        graph = torch.cuda.CUDAGraph()
        # thread_local: the RCCL watchdog thread of a multi-rank run keeps querying its events
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            for k in range(args.ring):
                vec.step(ring[k])
        graph.replay()  # untimed
        reps, rem = divmod(args.steps, args.ring)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            graph.replay()
        for k in range(rem):
            vec.step(ring[k])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        timing = f"hipGraph replay of {args.ring}-step segments"
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern_ms_max = float(t[0]), float(t[1])
    done_frac = float((vec.env_done != 0).float().mean())

    if rank == 0:
        total = world * e * n * args.steps
        value = total / wall
        bytes_launch = vec.algorithmic_bytes_per_step()
        achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
        wl = f"kinematic+swarm N={n} E={e}{' noterm' if args.no_term else ''}"
        rec = {
            "metric": METRIC, "value": value, "unit": "agent-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
            "ms_per_step_eager": wall_eager / args.steps * 1e3, "step_timing": timing,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (device-RNG episodes, uniform(-1,1) actions)",
            "config": {"workload": f"N={n} drones x E={e} envs per GPU, kinematic dynamics + "
                                   f"swarm reward, in-kernel auto-reset"
                                   f"{', no-termination radii' if args.no_term else ''}",
                       "num_drones": n, "envs_per_gpu": e, "global_envs": world * e,
                       "obs_dim": vec.obs_dim, "parallelism": f"env-sharded x{world}",
                       "ctde_allgather": bool(args.ctde and world > 1)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc_traffic(wl),
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "kernel_ms_mean": kern_ms, "kernel_ms_mean_max_rank": kern_ms_max,
                         "kernel": vec.kernel_name(),
                         "grid": int(vec.launch_info.blocks) if vec.persistent else e,
                         "timing": "HIP events on the launch stream around each step"},
            "env_done_fraction_last_step": done_frac,
        }
        if not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline(raw, n, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
