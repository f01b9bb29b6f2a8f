#!/usr/bin/env python3
"""Headline benchmark: agent-steps/s of the fused swarm step at N=64 drones x E=8192 envs/GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config headline|n16|n256]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N` alone (no WORLD_SIZE in the environment) makes this process a launcher: it spawns N
rank processes of this file, one per GPU, before touching the GPU itself, forwards rank 0's JSON
line and fails if any rank fails.  Under torchrun WORLD_SIZE must equal --gpus.  Fewer visible GPUs
than ranks is an error (SWARM_BENCH_REHEARSAL=1 shares cuda:0 over gloo; SWARM_BENCH_STANDIN=cpu
runs the rank plumbing with a CPU stand-in step, for the CPU tests).  The line carries the process
group's `world_size` and every rank's device (`rank_devices`).

One step = one launch of the fused kernel over the local env shard (integrate, distances,
collision, formation, rewards, terminations, in-kernel auto-reset, kNN obs) with inputs resident
in HBM.  Envs are sharded across ranks with no collective on the step path (weak scaling:
`--envs` envs per GPU, rank r owns the global envs [r*E, (r+1)*E)).

Timing (the driver's contract): W untimed warm-up steps, then exactly K timed steps bracketed by
a barrier + device synchronize on both sides, the max over ranks (each rank's clock runs from the
opening synchronize to the closing one).  The ranks' process group is gloo (barriers, the max)
unless `--ctde` gathers over RCCL: a rank without a data exchange holds no RCCL communicator.
K > 256 steps are replayed from a hipGraph holding one launch per action tensor of the ring (`value`, `ms_per_step`: the whole-job
rate without per-step host launch cost); short regions (the driver's K = 20) are launched eagerly
(host launches run ahead of the GPU; a replayed graph's kernels measured slower there); HIP events recorded on the launch stream around that
timed region give the average launch duration (`roofline.kernel_ms_mean`, the roofline's time
base; compare `rocprofv3 --kernel-trace --stats` in profiles/).  A second, eager pass with one
event pair per launch is reported as `ms_per_step_eager` / `kernel_ms_eager_events`.
`--ctde` also emits the CTDE global_state and, with several ranks, all-gathers it every
`--gather-every` steps over RCCL on a side stream, overlapped with the following steps (a
`--gs-slots` device ring; swarm_marl_amd.distributed.GlobalStateGather; config 5; eager timing).
Under SWARM_BENCH_REHEARSAL (gloo, every rank on cuda:0) the gather is staged through host memory.

`cpu_baseline` = the C port of the reference step (oracle/swarm_oracle.c) on the host cores for
a bounded sample of the same workload; `cpu_baseline_variants` = the per-agent loop restatement
(like the reference `DroneSwarmEnv.step`) and the vectorised NumPy restatement, one process per
core.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
sys.path.insert(0, str(ROOT))

METRIC = "agent-steps/sec at N=64 × E=8192 envs, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak in instruction-lanes/s: a wave64 VALU instruction occupies its SIMD-32 for 2
# cycles (MI355X_MICROARCH.md "Wave scheduling" and the v_fma_f32 row: 2 cyc throughput; the 4 cycles
# is what ONE wave alone sustains), so 32 lanes/clk/SIMD x 1024 SIMDs x 2.4 GHz.  SQ_INSTS_VALU x 64
# counts instruction-lanes.  (Rounds 2-4 priced 4 cycles, 39.3e12, which doubled the VALU fraction.)
VALU_PEAK_LANE_OPS = 78.6e12
# dense MFMA peaks, MI355X_MICROARCH.md; f32x3 runs three f16 MFMA passes per f32 product, so the
# f32-graph FLOPs it can deliver peak at a third of the f16 (= bf16) rate
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3, "f32x3": 2500.0 / 3}

# BASELINE.json configs, per GPU: [2] is the headline (the metric's config), [1] and [4] have
# their own bench lines (profiles/r02_config_lines.jsonl).
PRESETS = {
    "headline": dict(drones=64, envs=8192, ctde=False, groups=3, groups_graph=4,
                     label="config 3: N=64 x E=8192 on 1 MI355X (headline); config 4 per GPU"),
    # config 2 keeps graph replay for K > 256: 5.74-5.86 us per step on four boxes, while eager
    # launches of its 5.5 us kernel are bound by the host's launch rate, 5.47-6.84 us box to box
    # (profiles/r05u, r05x, r05y, r05z)
    "n16": dict(drones=16, envs=1024, ctde=False,
                label="config 2: N=16 x E=1024 on 1 MI355X (launch-latency-bound)"),
    "n256": dict(drones=256, envs=1024, ctde=True, groups=2, groups_graph=4,
                 label="config 5 per-GPU slab: N=256 x E=1024 with CTDE global_state"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", choices=sorted(PRESETS), default="headline")
    ap.add_argument("--drones", type=int, default=None)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU")
    ap.add_argument("--dynamics", choices=("kinematic", "physics"), default="kinematic",
                    help="physics = the point-mass restatement of DronePhysicsEnv (parity unpinned)")
    ap.add_argument("--no-term", action="store_true",
                    help="no-termination variant (collision/goal radii 0)")
    ap.add_argument("--ring", type=int, default=8, help="distinct pre-generated action tensors")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="timed seconds of the C-port CPU baseline")
    ap.add_argument("--cpu-variant-seconds", type=float, default=3.0,
                    help="timed seconds of each Python restatement variant (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--waves-per-simd", type=int, default=0,
                    help="persistent step kernel: resident waves per SIMD (0 = library default)")
    ap.add_argument("--no-persistent", action="store_true",
                    help="one workgroup per env instead of the persistent env queue")
    ap.add_argument("--no-graph", action="store_true",
                    help="time the whole-job rate with eager launches instead of hipGraph replay")
    ap.add_argument("--ctde", action="store_true", default=None,
                    help="also emit global_state and all-gather it (config 5)")
    ap.add_argument("--no-ctde", dest="ctde", action="store_false",
                    help="no global_state output (the n256 preset emits it by default)")
    ap.add_argument("--eval", action="store_true",
                    help="on-device eval metrics every step (EvalTracker: swarm_eval_update per env group "
                         "after its step; the envs carry infos): the evaluation-protocol rollout")
    ap.add_argument("--policy", choices=("bf16", "f32", "f32x3"), default=None,
                    help="rollout mode: each step = on-device actor inference on the obs tensor "
                         "(swarm_policy_forward, random-init TorchFC 256x256 weights) + the env step")
    ap.add_argument("--device-warmup-ms", type=float, default=200.0,
                    help="untimed graph replays for this long before the timed region, after the W "
                         "warm-up steps (GPU clocks ramp over ~100 ms; reported in the JSON line)")
    ap.add_argument("--groups", type=int, default=None,
                    help="env groups per GPU, each stepped on its own HIP stream (VecSwarm groups=G); "
                         "default: 4 with graph replay (K > 256), else the preset's (headline 3, n256 2); 1 for n16")
    ap.add_argument("--graph", choices=("split", "fused"), default="split",
                    help="env groups in the timed hipGraph: one graph per group stream, or one graph "
                         "holding every group's chain (fork/join captured)")
    ap.add_argument("--rehearse", type=int, default=3,
                    help="untimed runs of the whole K-step region (each between device syncs) after the "
                         "device warm-up, so the timed region follows what it would follow in a loop "
                         "of such regions, not a 200 ms burst (round 3: the first region after the burst ran "
                         "28.5-29.9 us per step, repeats 26.0-28.0)")
    ap.add_argument("--region-reps", type=int, default=1,
                    help="diagnostic: time the K-step region this many times back to back; the line "
                         "reports the first, `ms_per_step_reps` lists all")
    ap.add_argument("--events-before", type=int, default=1,
                    help="eager regions: record the device-time start events before the opening synchronize "
                         "(1) instead of as the region's first calls (0).  The wall clock is unchanged; the "
                         "device span then also holds the gap from the synchronize to the first launch "
                         "(r04e, driver command x3 each: 25.39 vs 26.17 us per step)")
    ap.add_argument("--spin-sync", action="store_true",
                    help="diagnostic: poll the closing event before the closing synchronize")
    ap.add_argument("--graph-short", action="store_true",
                    help="replay hipGraphs for short timed regions too (K <= 256; default there: eager launches)")
    ap.add_argument("--eager-head", type=int, default=0,
                    help="short timed regions (K <= 256): launch the first H steps eagerly, then replay a graph "
                         "of the remaining K - H (the GPU starts while the host launches the graph)")
    ap.add_argument("--warm-graph", choices=("whole", "ring"), default="whole",
                    help="device warm-up replays the timed K-step graph (whole) or the 8-step ring graphs")
    ap.add_argument("--split-reset", action="store_true",
                    help="diagnostic: after each group launch, swarm_reset of the envs it reset (timing only)")
    ap.add_argument("--stagger-us", type=float, default=0.0,
                    help="diagnostic: group 1's first timed step starts this much later (phase offset)")
    ap.add_argument("--gather-every", type=int, default=8,
                    help="CTDE all-gather period in steps (SURVEY.md §5: per batch, not per step)")
    ap.add_argument("--graph-gather", action="store_true",
                    help="CTDE gathering runs with K > 256 and --gather-every = --ring replay graphs of ring-step "
                         "segments (two slot halves of a 2 x ring slot ring, the gather between segment replays); "
                         "default eager: with an RCCL communicator in the process the replays ran slower "
                         "(config 5: 42.3-45.4 vs 39.9 us per step, profiles/r06q_graph_gather_ab.jsonl)")
    ap.add_argument("--gs-slots", type=int, default=4,
                    help="CTDE global_state ring slots (multi-rank): a gathered slot is rewritten "
                         "only R steps later, so the gather overlaps R-1 steps")
    a = ap.parse_args(argv)
    pre = PRESETS[a.config]
    a.drones = pre["drones"] if a.drones is None else a.drones
    a.envs = pre["envs"] if a.envs is None else a.envs
    a.ctde = pre["ctde"] if a.ctde is None else a.ctde
    a.label = pre["label"]
    a.groups_explicit = a.groups is not None
    if a.groups is None:
        # 4 groups where the timed region replays graphs (K > 256, no CTDE gather): 25.2 vs
        # 26.7 us (headline), 56.2 vs 61.0 us (n256); eager short regions (the driver's K = 20)
        # use the preset's `groups`: headline 3 (one native call launches them; 3 group streams +
        # the default stream fit GPU_MAX_HW_QUEUES = 4): 24.88 vs 25.18 us for 2 over 8 + 8
        # alternating runs (profiles/r04s_groups.txt; 4 groups 25.3-25.4, 1 group 29.2-29.3)
        gathering = a.ctde and (int(os.environ.get("WORLD_SIZE", "1")) > 1
                                or os.environ.get("SWARM_BENCH_FORCE_GATHER") == "1")
        graph_long = (a.steps > 256 and not a.no_graph and not a.eval
                      and (not gathering or (a.graph_gather and a.gather_every == a.ring)))
        a.groups = pre.get("groups_graph", pre.get("groups", 1)) if graph_long else pre.get("groups", 1)
        if not graph_long and gathering and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # a gathering rank also holds RCCL's streams and the gather's side stream: 2 group
            # streams + the default stream + RCCL stay within GPU_MAX_HW_QUEUES = 4.  Ranks without
            # the gather hold no RCCL communicator (main(): gloo) and keep the one-rank groups
            a.groups = min(a.groups, 2)
    if a.groups < 1:
        ap.error("--groups must be >= 1")

    if a.gather_every < 1:
        ap.error("--gather-every must be >= 1")
    if a.gs_slots < 1:
        ap.error("--gs-slots must be >= 1")
    return a


# ----------------------------------------------------------------------------- rank logic
def shard_plan(world: int, rank: int, envs_per_gpu: int) -> tuple[int, int]:
    """(env_offset, count) of `rank`: weak scaling, each rank owns envs_per_gpu global envs."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return rank * envs_per_gpu, envs_per_gpu


def max_over_ranks(values, world: int, device=None) -> list[float]:
    """Element-wise MAX of per-rank floats (a tiny all_reduce outside the timed region)."""
    import torch
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if world > 1:
        import torch.distributed as dist
        if dist.get_backend() == "gloo":  # rehearsal backend: host tensors
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def pg_backend(ctde: bool, rehearsal: bool) -> str:
    """Process-group backend of a multi-rank run: RCCL ("nccl") only for the CTDE gather on real
    GPUs; gloo for the barriers and the max over ranks otherwise (and for the rehearsal)."""
    return "nccl" if ctde and not rehearsal else "gloo"


def _barrier_on(world: int) -> bool:
    if world > 1:
        return True
    import torch.distributed as dist
    return os.environ.get("SWARM_BENCH_ONE_RANK_PG", "") in ("1", "nccl", "gloo") and dist.is_initialized()


def timed_region(body, world: int, sync, spin=None, pre=None) -> float:
    """Barrier + sync, run `body`, sync + barrier; wall seconds of this rank from the opening sync
    to the closing sync (the caller takes the max over ranks: every rank starts after the common
    barrier, so the max is the job's time; the closing barrier's own latency, ~25-40 us over gloo
    and more over RCCL, is not step time: profiles/r06m_pg_backend_ab.jsonl).  `spin`: an event
    polled until it completes before the closing sync (diagnostic --spin-sync).  `pre`: run
    before the opening sync (the start events of the device-time bracket: their host cost would
    otherwise delay the region's first launch)."""
    if _barrier_on(world):
        import torch.distributed as dist
        dist.barrier()
    if pre is not None:
        pre()
    sync()
    t0 = time.perf_counter()
    body()
    if spin is not None:
        while not spin.query():
            pass
    sync()
    t1 = time.perf_counter()
    if _barrier_on(world):
        import torch.distributed as dist
        dist.barrier()
    return t1 - t0


def gather_schedule(steps: int, every: int) -> list[int]:
    """Timed-step indices after which the CTDE all-gather runs (every `every` steps + the last)."""
    ks = [k for k in range(steps) if (k + 1) % every == 0]
    if steps and (not ks or ks[-1] != steps - 1):
        ks.append(steps - 1)
    return ks


# ----------------------------------------------------------------------------- CPU baselines
def _cpu_cores() -> tuple[int, str]:
    """Host cores this process may use: the affinity set, capped by OMP_NUM_THREADS when the
    harness sets it to the box's CPU share (os.cpu_count() shows the whole machine there)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"{omp} threads = OMP_NUM_THREADS (this host's CPU share; {aff} in the affinity set)"
    return aff, f"{aff} threads = every core of the affinity set"


def cpu_baseline_port(n: int, e: int, seconds: float, raw: dict, physics: bool = False) -> dict:
    """C port of the reference step (oracle/swarm_oracle.c, OpenMP) on the benched workload:
    same N and E, auto-reset on, persistent buffers, a bounded number of steps."""
    from oracle import c_oracle as co
    from oracle import swarm_oracle as so

    cores, why = _cpu_cores()
    cfg = so.make_cfg(**raw)
    run = co.Runner(cfg, e, seed=0, nthreads=cores, physics=physics)
    rng = np.random.default_rng(1000)
    ring = [rng.uniform(-1, 1, (e, n, 3)).astype(np.float32) for _ in range(4)]
    run.step(ring[0])  # warm
    steps, t0 = 0, time.perf_counter()
    while True:
        run.step(ring[steps % 4])
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": e * n * steps / el, "unit": "agent-steps/s", "cores": cores, "kind": "port",
            "sample": f"C port of {'DronePhysicsEnv (point-mass restatement)' if physics else 'DroneSwarmEnv'}"
                      f".step (oracle/swarm_oracle.c), OpenMP {why}; "
                      f"N={n} x E={e} envs (the benched workload), {steps} steps in {el:.2f} s, "
                      f"auto-reset on, " + ("bit-identical to the GPU kernel (physics parity unpinned)" if physics
                                            else "bit-exact with the reference fixtures")}


def cpu_python_variants(n: int, e: int, seconds: float, procs: int | None = None) -> list[dict]:
    """BASELINE.md §5 (a) per-agent loop restatement and (b) vectorised NumPy restatement, one
    single-threaded process per core with the envs split across them."""
    if procs is None:
        procs, _ = _cpu_cores()
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1",
               PYTHONPATH=os.pathsep.join([str(ROOT), os.environ.get("PYTHONPATH", "")]))
    out = []
    for kind, desc in (("loop", "per-agent loop restatement (oracle/swarm_loop.py, the reference "
                                "DroneSwarmEnv.step's structure)"),
                       ("numpy", "vectorised NumPy restatement (oracle/swarm_oracle.py)")):
        per = max(1, e // procs) if kind == "numpy" else max(1, min(4, e // procs))
        ps = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_bench", "--kind", kind,
                                "--drones", str(n), "--envs", str(per), "--seconds", str(seconds),
                                "--seed", str(k)], stdout=subprocess.PIPE, cwd=str(ROOT), env=env)
              for k in range(procs)]
        res = []
        for p in ps:
            so_, _ = p.communicate(timeout=seconds * 20 + 120)
            if p.returncode != 0:
                raise RuntimeError(f"cpu_bench {kind} failed ({p.returncode})")
            res.append(json.loads(so_.decode().strip().splitlines()[-1]))
        total = sum(r["agent_steps"] for r in res)
        el = max(r["seconds"] for r in res)
        out.append({"value": total / el, "unit": "agent-steps/s", "cores": procs, "kind": "port",
                    "sample": f"{desc}: {procs} single-threaded processes x {per} envs of N={n}, "
                              f"{total} agent-steps in {el:.2f} s, auto-reset on"})
    return out


# ----------------------------------------------------------------------------- profile data
def profile_record(workload_key: str):
    """Counter data for this workload from the committed rocprofv3 PMC summary (not measured in
    this run): HBM bytes per launch and VALU instructions per launch."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(workload_key)
    except Exception:
        return None


def valu_roofline(prof: dict, kern_ms: float) -> dict:
    """VALU side of the roofline from the committed PMC record of this workload (not measured in
    this run) against this run's step time `kern_ms` (one step = every env of the GPU once):
    * frac_2cycle: SQ_INSTS_VALU x 64 lanes against VALU_PEAK_LANE_OPS (every instruction at the
      full, 2-cycle rate): a LOWER bound, since about half of the step's instructions are
      half-rate encodings (min / max / med3, packed f32, DPP, compares, f64, conversions);
    * busy_class_costed [lo, hi]: per-SIMD VALU issue time (the PMC instruction classes priced at
      their cheapest / dearest member's measured ns per wave-instruction per SIMD, tools/valu_busy.py,
      profiles/r05o_valu_rate4.txt) / step time; busy_frac = hi (the occupancy sweep's measured
      marginal cost per wave, DESIGN.md §6, lands at the top of the bracket);
    * counter_frac: 4 x SQ_ACTIVE_INST_VALU (quad-cycles per wave, summed over the step's waves)
      / (SIMDs x step time x 2.4 GHz) — the counter charges one quad-cycle per VALU instruction,
      so it reads as a 4-cycle model at the nominal clock."""
    lane_ops = prof["valu_insts_per_launch"] * 64.0
    out = {"frac_2cycle": lane_ops / (kern_ms * 1e-3) / VALU_PEAK_LANE_OPS,
           "achieved_lane_ops_per_s": lane_ops / (kern_ms * 1e-3), "peak_lane_ops_per_s": VALU_PEAK_LANE_OPS,
           "frac_2cycle_note": "lower bound: SQ_INSTS_VALU x 64 lanes at 32 lanes/clk/SIMD (a wave64 "
                               "instruction at the full 2-cycle rate) x 1024 SIMDs x 2.4 GHz",
           "valu_insts_per_wave": prof.get("valu_insts_per_wave")}
    waves, simds = prof.get("waves"), prof.get("simds", 1024)
    ns = prof.get("valu_issue_ns_per_wave")
    if waves and ns:
        per_simd_us = [x * waves / simds * 1e-3 for x in ns]
        out["valu_issue_us_per_simd_per_step"] = [round(x, 3) for x in per_simd_us]
        out["busy_class_costed"] = [x / (kern_ms * 1e3) for x in per_simd_us]
        out["busy_frac"] = out["busy_class_costed"][1]
    act = prof.get("active_inst_valu_per_wave")
    if waves and act:
        out["counter_frac"] = 4.0 * act * waves / simds / (kern_ms * 1e-3 * 2.4e9)
    out["source"] = (f"profiles/pmc_traffic.json (rounds {prof.get('round')} / {prof.get('valu_class_round')}); "
                     "class prices from profiles/r05o_valu_rate4.txt; python tools/valu_busy.py "
                     f"{prof.get('valu_class_round')} reproduces the per-wave figures")
    return out


# ----------------------------------------------------------------------------- main
def main(argv=None):
    import torch
    import torch.distributed as dist

    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SWARM_BENCH_REHEARSAL=1: every rank on cuda:0 with the gloo backend — the multi-rank code
    # path (sharding, barriers, max-reduce) rehearsed on a one-GPU box; not a scaling measurement
    rehearsal = os.environ.get("SWARM_BENCH_REHEARSAL") == "1"
    if world > 1:
        if not rehearsal:
            if torch.cuda.device_count() < world:  # the launcher parent did not open the GPU to check
                raise SystemExit(f"bench.py rank {rank}: {world} ranks need {world} GPUs (one per rank), "
                                 f"{torch.cuda.device_count()} visible")
            torch.cuda.set_device(local)
        # RCCL only where the step path exchanges data (the CTDE global_state all-gather); otherwise
        # the barriers and the max over ranks go over gloo: a process holding an RCCL communicator ran
        # the driver's command 27.0-28.8 us per step against 24.5-25.2 without one (r06m, one-rank
        # groups; the launches reach and leave the queues more slowly, 8 hardware queues do not help:
        # DESIGN.md §7, r06o-r06r)
        dist.init_process_group(pg_backend(args.ctde, rehearsal))
    dev = torch.device("cuda", local if world > 1 and not rehearsal else 0)
    torch.cuda.set_device(dev)
    own_pg = False
    # SWARM_BENCH_ONE_RANK_PG=nccl|gloo (diagnostic; 1 = nccl): a one-rank process group whose barrier
    # brackets the timed region, so a one-GPU box sees what a multi-rank process holds
    # (profiles/r06l_groups_rccl_ab.jsonl, r06m / r06n_pg_backend_ab.jsonl)
    one_rank_pg = world == 1 and os.environ.get("SWARM_BENCH_ONE_RANK_PG", "") in ("1", "nccl", "gloo")
    if world == 1 and (one_rank_pg or (os.environ.get("SWARM_BENCH_FORCE_GATHER") == "1" and args.ctde)) \
            and not dist.is_initialized():
        # the CTDE gather on one GPU: a one-rank RCCL group (its cost on the step)
        import socket
        with socket.socket() as so_:
            so_.bind(("127.0.0.1", 0))
            port = so_.getsockname()[1]
        backend = "gloo" if one_rank_pg and os.environ["SWARM_BENCH_ONE_RANK_PG"] == "gloo" else "nccl"
        # SWARM_BENCH_PG_EAGER=1 (diagnostic): the RCCL communicator (and its streams) created here,
        # before the env's group streams, instead of at the first collective
        eager = {"device_id": dev} if backend == "nccl" and os.environ.get("SWARM_BENCH_PG_EAGER") == "1" else {}
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, **eager)
        own_pg = True

    from swarm_marl_amd import VecSwarm

    n = args.drones
    offset, e = shard_plan(world, rank, args.envs)
    # SWARM_BENCH_FORCE_GATHER=1: run the gather with a one-rank process group the caller set
    # up (tests/test_gpu_ctde.py drives this branch over RCCL on one GPU)
    gathering = args.ctde and (world > 1 or (os.environ.get("SWARM_BENCH_FORCE_GATHER") == "1"
                                             and dist.is_initialized()))
    # --graph-gather: a gathering run with a long timed region replays graphs too: two sets of ring-step segment
    # graphs, each writing its own half of a 2 x ring slot global_state ring, and the gather of a
    # segment's last slot issued between segment replays (overlapping the next segment; the segment
    # after that, which rewrites the slot, waits for it)
    args.graph_gather = (args.graph_gather and gathering and args.steps > 256 and not args.no_graph
                         and not args.eval and not args.policy and args.gather_every == args.ring)
    if args.graph_gather:
        args.gs_slots = 2 * args.ring
    raw = {"num_drones": n}
    if args.no_term:
        raw.update(collision_radius=0.0, obstacle_radius=0.0, goal_radius=0.0)
    vec = VecSwarm(e, raw, device=dev, auto_reset=True, seed=0, env_offset=offset, dynamics=args.dynamics,
                   with_global_state=args.ctde, persistent=not args.no_persistent,
                   waves_per_simd=args.waves_per_simd, groups=args.groups,
                   global_state_slots=args.gs_slots if gathering else 1, with_infos=args.eval)
    vec.reset()
    tracker = None
    if args.eval:
        from swarm_marl_amd.eval_metrics import EvalTracker
        tracker = EvalTracker(vec, capacity=1 << 20)  # later episodes past a full segment are dropped
        tracker.begin()
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    ring = [torch.rand((e, n, 3), device=dev, generator=gen) * 2 - 1 for _ in range(args.ring)]
    pol, pol_act = None, None
    if args.policy:
        from swarm_marl_amd.policy import PolicyMLP
        rng = np.random.default_rng(7)  # random-init weights of the reference architecture
        d = vec.obs_dim
        pol = PolicyMLP.from_arrays(rng.normal(0, d ** -0.5, (256, d)), np.zeros(256),
                                    rng.normal(0, 256 ** -0.5, (256, 256)), np.zeros(256),
                                    rng.normal(0, 0.01, (6, 256)), np.zeros(6), device=dev,
                                    precision=args.policy)
        pol_act = torch.zeros((e, n, 3), device=dev)
    gatherer = None
    gathers = set()
    if gathering:
        # CTDE: every step writes global_state into slot k % R of a device ring; the gather
        # steps' slots are all-gathered on a side stream while the next steps run (RCCL; the
        # gloo rehearsal stages through pinned host memory), distributed.GlobalStateGather
        from swarm_marl_amd.distributed import GlobalStateGather
        gatherer = GlobalStateGather(vec.global_state_ring, vec.select_global_state_slot)
        gathers = set(gather_schedule(args.steps, args.gather_every))

    G = vec.groups
    slices = vec.group_slices

    import ctypes

    def split_reset(g):  # diagnostic (--split-reset): the group's reset envs by swarm_reset
        lo = slices[g][0]
        vec.lib.swarm_reset(ctypes.byref(vec._gparams[g]), ctypes.byref(vec._gstate[g]),
                            vec.env_done.data_ptr() + lo, ctypes.byref(vec._gout[g]), vec._stream())

    def env_step_group(g, k):  # group g's step k on the current stream
        if pol is not None:  # rollout: actions from the policy on the current obs, in place
            lo, hi = slices[g]
            pol.act(vec.obs[lo:hi], out=pol_act[lo:hi])
            vec.step_group(g, pol_act)
        else:
            vec.step_group(g, ring[k % args.ring])
        if tracker is not None:
            tracker.update_group(g)
        if args.split_reset:
            split_reset(g)

    # plain env steps with groups: one native call launches every group on its stream
    # (swarm_step_groups), instead of a Python stream context + launch per group
    # (a fused eval tracker needs no launch of its own: the step launches update it)
    native_groups = G > 1 and pol is None and (tracker is None or tracker.fused) and not args.split_reset

    def env_step(k):  # whole batch: group g on group stream g (not joined: groups overlap)
        if G == 1:
            env_step_group(0, k)
            return
        if native_groups:
            vec.step_groups(ring[k % args.ring])
            if tracker is not None:
                tracker.update()
            return
        for g, st in enumerate(vec.group_streams):
            with torch.cuda.stream(st):
                env_step_group(g, k)

    launch_streams = vec.group_streams if G > 1 else [torch.cuda.current_stream(dev)]

    def step(k):
        if gatherer is None:
            env_step(k)
            return
        gatherer.before_step(launch_streams)
        env_step(k)
        gatherer.after_step(launch_streams, gather=k in gathers)

    stream = torch.cuda.current_stream(dev)
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    sync()  # the reset and the action ring are done before any group stream steps
    for k in range(args.warmup):
        step(k)
    sync()

    # With env groups the timed region is bracketed on group stream 0 (the other groups fork
    # from and join into it): the null stream, which may share a hardware queue with a group
    # stream, then carries no work inside the timed region.
    if G > 1:
        stream = vec.group_streams[0]

    def fork(ev):  # the other group streams start after `ev` on the bracket stream
        if G > 1:
            for st in vec.group_streams[1:]:
                st.wait_event(ev)

    def join():
        if G > 1:
            for st in vec.group_streams[1:]:
                stream.wait_stream(st)
        if gatherer is not None and gatherer.stream is not None:  # the region ends after the last gather
            stream.wait_stream(gatherer.stream)

    # ---- timed region: hipGraph replay of ring segments (or eager with --no-graph / CTDE)
    # With env groups: one graph per group, captured and replayed on its group stream; the
    # events on the launch stream fork to / join from the group streams, so they bracket the
    # whole batch's K steps.
    t_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    # short timed regions (the driver's K = 20) launch eagerly: a replayed graph's kernels ran
    # slower there (27.5-28.8 vs 30.8-32.3 us per step by events, round 3); graphs for
    # long regions, where the host's ~5 us per launch would otherwise matter
    # --eval launches eagerly: a captured swarm_eval_update would replay its capture-time update
    # index, so the records' update order and the update count would be wrong
    use_graph = args.graph_gather or (not args.no_graph and gatherer is None and tracker is None
                                      and (args.steps > 256 or args.graph_short))
    reps, rem = divmod(args.steps, args.ring)
    if use_graph:
        def capture(n_steps, k0=0, slots=False):  # one graph of n_steps ring steps per group, on its group stream
            out = []
            for g in range(G):
                gr = torch.cuda.CUDAGraph()

                def seg():
                    for k in range(k0, k0 + n_steps):
                        if slots:  # step k writes global_state slot k mod 2 x ring (baked into the graph)
                            vec.select_global_state_slot(k % args.gs_slots)
                        env_step_group(g, k)
                # thread_local: the RCCL watchdog thread of a multi-rank run keeps querying its events
                if G == 1:
                    with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                        seg()
                else:
                    st = vec.group_streams[g]
                    with torch.cuda.stream(st), torch.cuda.graph(gr, stream=st, capture_error_mode="thread_local"):
                        seg()
                out.append(gr)
            return out
        def capture_fused(n_steps):  # ONE graph holding every group's chain (fork / join inside)
            gr = torch.cuda.CUDAGraph()
            s0 = vec.group_streams[0]
            with torch.cuda.stream(s0), torch.cuda.graph(gr, stream=s0, capture_error_mode="thread_local"):
                ev_f = torch.cuda.Event()
                ev_f.record(s0)
                for st in vec.group_streams[1:]:
                    st.wait_event(ev_f)
                for k in range(n_steps):
                    for g, st in enumerate(vec.group_streams):
                        with torch.cuda.stream(st):
                            env_step_group(g, k)
                for st in vec.group_streams[1:]:
                    ev_j = torch.cuda.Event()
                    ev_j.record(st)
                    s0.wait_event(ev_j)
            return [gr]

        fused = args.graph == "fused" and G > 1 and not args.graph_gather
        if args.graph_gather:
            # the gatherer's step count must sit on a slot-ring boundary when segment replays start:
            # untimed eager steps without gathers up to it
            while gatherer.k % args.gs_slots:
                gatherer.before_step(launch_streams)
                env_step(gatherer.k)
                gatherer.after_step(launch_streams, gather=False)
            sync()
            halves = [capture(args.ring, 0, slots=True), capture(args.ring, args.ring, slots=True)]
            vec.select_global_state_slot(0)
        graphs = capture(args.ring) if not args.graph_gather else halves[0]
        # short timed regions (the driver's K = 20) replay all K steps from one graph per group
        # (or one fused graph), so that the wall clock holds one graph launch per group; longer
        # ones replay ring segments plus a graph of the K % ring remainder
        head = max(0, min(args.eager_head, args.steps - 1)) if args.steps <= 256 and not fused else 0
        whole = (capture_fused(args.steps) if fused else capture(args.steps - head, head)) \
            if args.steps <= 256 and not args.graph_gather else None
        tail = capture(rem) if rem and whole is None and not args.graph_gather else None

        def replay_all(gs):
            if G == 1 or len(gs) == 1:  # one group, or the fused graph (on group stream 0)
                with torch.cuda.stream(stream if G == 1 else vec.group_streams[0]):
                    gs[0].replay()
                return
            for g, st in enumerate(vec.group_streams):
                with torch.cuda.stream(st):
                    gs[g].replay()
        def gather_segments(k0, n_seg):  # graph-gather mode: n_seg segment replays from timed step k0
            for j in range(n_seg):
                ks = range(k0 + j * args.ring, k0 + (j + 1) * args.ring)
                # the group streams wait for the gathers of the slot half this segment rewrites
                gatherer.before_steps(args.ring, launch_streams)
                replay_all(halves[(gatherer.k // args.ring) % 2])
                for k in ks:
                    gatherer.after_step(launch_streams, gather=k in gathers)

        if args.graph_gather:
            gather_segments(-(1 << 30), 2)  # untimed, no gathers (k < 0): each half launched once
        else:
            replay_all(graphs)  # untimed
        if whole is not None:
            replay_all(whole)  # untimed: the timed region is not the graph's first launch
        sync()

        def body():
            t_ev[0].record(stream)
            if not (fused and whole is not None):
                fork(t_ev[0])
            if args.stagger_us > 0 and G > 1:  # diagnostic: start group 1 later (phase offset)
                with torch.cuda.stream(vec.group_streams[1]):
                    torch.cuda._sleep(int(args.stagger_us * 2400))
            if args.graph_gather:
                gather_segments(0, reps)
                for k in range(reps * args.ring, args.steps):  # the K mod ring remainder, eager
                    step(k)
            elif whole is not None:
                for k in range(head):  # eager head: the first kernels start at once
                    env_step(k)
                replay_all(whole)
            else:
                for _ in range(reps):
                    replay_all(graphs)
                if tail is not None:
                    replay_all(tail)
            if not (fused and whole is not None):
                join()
            t_ev[1].record(stream)
        timing = ((f"{head} eager step(s), then " if head else "") +
                  f"hipGraph replay of the {args.steps - head} steps (actions from a {args.ring}-tensor ring)"
                  if whole is not None else f"hipGraph replay of {args.ring}-step segments") + (
            f", CTDE all-gather of each segment's last global_state slot between segment replays (a "
            f"{args.gs_slots}-slot ring, segments alternating halves; the K mod {args.ring} remainder eager)"
            if args.graph_gather else "") + (
            (f", {G} env groups on {G} HIP streams (" + ("one graph holding all groups" if fused and whole is not None
                                                        else "one graph per group") + ")") if G > 1 else "") + (
            f" (policy {args.policy} + env step per step)" if pol is not None else "") + (
            " + eval metrics update per group" if tracker is not None else "")
    else:
        # The device synchronise before t0 already orders the region after every earlier launch,
        # and the closing one waits for every stream: the group streams need no fork from / join
        # to a bracket stream (each costs the command processor a barrier packet per stream,
        # ~15 us per region, tools/k20_intercept.py).  Events on every group stream give the
        # device time.  A CTDE gather keeps the bracket stream (its side stream joins into it).
        free = gatherer is None and G > 1
        ev_free = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(G)] if free else []

        def start_events():
            if free:
                for (e0, _), st in zip(ev_free, vec.group_streams):
                    e0.record(st)
            else:
                t_ev[0].record(stream)
                fork(t_ev[0])

        def body():
            if not args.events_before:
                start_events()
            for k in range(args.steps):
                step(k)
            if free:
                for (_, e1), st in zip(ev_free, vec.group_streams):
                    e1.record(st)
            else:
                join()
                t_ev[1].record(stream)
        timing = "eager launches" + (f", {G} env groups on {G} HIP streams" if G > 1 else "") + (
            f", CTDE all-gather every {args.gather_every} steps from the default stream when no group launches there, else a side stream ({args.gs_slots}-slot "
            f"global_state ring{', gloo host-staged' if gatherer is not None and gatherer.staged else ''})"
            if gatherer is not None else "")
    # every event the region records exists before it: torch creates an event's HIP object at
    # its first record, which would otherwise land inside the timed region (the first region
    # after the warm-up measured 31.0 us per step against 26.4-28.1 for repeats, --region-reps)
    for e_ in list(t_ev) + ([e for pair in ev_free for e in pair] if not use_graph else []):
        e_.record(stream)
    sync()
    # device warm-up: untimed ring segments until the clocks have ramped (not part of W or K)
    warm_ms, warm_steps = 0.0, 0
    if args.device_warmup_ms > 0:
        sync()
        t0 = time.perf_counter()
        # time-based unless a step holds a collective (every rank must then run the same count)
        fixed = None if gatherer is None else max(args.ring, int(args.device_warmup_ms * 5))
        while ((time.perf_counter() - t0) * 1e3 < args.device_warmup_ms if fixed is None
               else warm_steps < fixed):
            if args.graph_gather:
                gather_segments(-(1 << 30), 1)
                warm_steps += args.ring
            elif use_graph:
                if whole is not None and args.warm_graph == "whole":
                    replay_all(whole)
                    warm_steps += args.steps
                else:
                    replay_all(graphs)
                    warm_steps += args.ring
            else:
                for k in range(args.ring):
                    step(k)
                warm_steps += args.ring
            if warm_steps % (8 * args.ring) == 0:
                sync()
        sync()
        warm_ms = (time.perf_counter() - t0) * 1e3
    pre = start_events if (not use_graph and args.events_before) else None
    if gatherer is None:
        for _ in range(max(0, args.rehearse)):
            timed_region(body, world, sync, pre=pre)
    gather_t0 = gatherer.k if gatherer is not None else 0
    wall = timed_region(body, world, sync, spin=t_ev[1] if args.spin_sync else None, pre=pre)
    walls_rep = [wall]
    for _ in range(args.region_reps - 1):  # diagnostic repeats (not reported as the value)
        walls_rep.append(timed_region(body, world, sync, pre=pre))
    if not use_graph and free:  # first start to last end over the group streams
        f0 = ev_free[0][0]
        kern_ms = (max(f0.elapsed_time(e1) for _, e1 in ev_free) -
                   min(f0.elapsed_time(e0) for e0, _ in ev_free)) / args.steps
    else:
        kern_ms = t_ev[0].elapsed_time(t_ev[1]) / args.steps

    # ---- diagnostic pass: eager launches, one event pair around every launch on its stream
    # (with env groups the launches of a step overlap: the per-launch mean is what rocprofv3
    # reports per dispatch, the whole pass / K is the eager step time)
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)] for _ in range(G)]
    ev_all = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    streams_g = vec.group_streams if G > 1 else [stream]

    raw_launch = native_groups  # plain steps: launch group g straight onto its stream handle

    def body_eager():
        ev_all[0].record(stream)
        fork(ev_all[0])
        for k in range(args.steps):
            for g, st in enumerate(streams_g):
                if raw_launch:
                    ev[g][k][0].record(st)
                    vec._launch_step(g, ring[k % args.ring], None, vec._gstream_h[g])
                    ev[g][k][1].record(st)
                    continue
                with torch.cuda.stream(st):
                    ev[g][k][0].record(st)
                    env_step_group(g, k)
                    ev[g][k][1].record(st)
        join()
        ev_all[1].record(stream)
    wall_eager = timed_region(body_eager, world, sync)
    kern_launch = float(np.mean([a.elapsed_time(b) for row in ev for a, b in row]))
    kern_eager = ev_all[0].elapsed_time(ev_all[1]) / args.steps

    pol_ms = 0.0
    if pol is not None:  # the policy kernel alone, K launches on the current obs, events around them
        pe = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        sync()
        cs = torch.cuda.current_stream(dev)
        pe[0].record(cs)
        for _ in range(args.steps):
            pol.act(vec.obs, out=pol_act)
        pe[1].record(cs)
        sync()
        pol_ms = pe[0].elapsed_time(pe[1]) / args.steps
    wall_max, kern_max, eager_max, kern_eager_max, launch_max, pol_max = max_over_ranks(
        [wall, kern_ms, wall_eager, kern_eager, kern_launch, pol_ms], world, dev)
    done_frac = float((vec.env_done != 0).float().mean())
    props = torch.cuda.get_device_properties(dev)
    devs = rank_devices(world, {"rank": rank, "local_rank": local, "device": int(dev.index),
                                "name": props.name, "pci_bus_id": getattr(props, "pci_bus_id", None),
                                "uuid": str(getattr(props, "uuid", "")) or None, "env_offset": offset})
    world_pg = dist.get_world_size() if (world > 1 and dist.is_initialized()) else 1
    if world_pg != world:
        raise RuntimeError(f"process group holds {world_pg} ranks, WORLD_SIZE {world}")
    if world > 1 and not rehearsal and len({(d["device"], d["pci_bus_id"], d["uuid"]) for d in devs}) < world:
        raise RuntimeError(f"ranks share a GPU (one rank per GPU expected): {devs}")

    if rank == 0:
        total = world * e * n * args.steps
        value = total / wall_max
        bytes_launch = vec.algorithmic_bytes_per_step()
        achieved = bytes_launch / (kern_max * 1e-3) / 1e9
        wl = ("kinematic+swarm" if args.dynamics == "kinematic" else "physics") + \
             f" N={n} E={e}{' noterm' if args.no_term else ''}" + \
             (" +global_state" if args.ctde else "")
        prof = profile_record(wl) or {}
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": prof.get("hbm_bytes_per_launch"),
                "traffic_source": (f"rocprofv3 PMC (2 x FETCH_SIZE + WRITE_SIZE) of this workload, "
                                   f"profiles/pmc_traffic.json round {prof.get('round')}; not "
                                   f"measured in this run") if prof else None,
                "algorithmic_bytes_per_launch": bytes_launch,
                "kernel_ms_mean": kern_max,
                "kernel_ms_timing": (f"HIP events on the launch stream around the timed region "
                                     f"({'graph replays' if use_graph else 'eager launches'}), / K; max over ranks")
                                    if G == 1 else
                                    (f"HIP events on every group stream around the timed region (eager "
                                     f"launches): last end - first start, / K = whole-batch step time "
                                     f"({G} overlapping launches of E/{G} envs per step); max over ranks")
                                    if not use_graph and free else
                                    (f"HIP events on the launch stream around the timed region, "
                                     f"forked to and joined from the {G} group streams ("
                                     f"{'graph replays' if use_graph else 'eager launches'}), / K = whole-batch "
                                     f"step time ({G} overlapping launches of E/{G} envs per step); max over ranks"),
                "kernel_ms_eager_events": kern_eager_max,
                "kernel_ms_per_launch": launch_max,
                "kernel_ms_per_launch_timing": "eager pass, HIP events around each launch on its own "
                                               "stream, mean (compare rocprofv3 per-dispatch average"
                                               + (f"; the {G} launches of a step overlap" if G > 1 else "") + ")",
                "kernel": vec.kernel_name(),
                "grid": int(vec.group_launch_info[0].blocks),
                "env_groups": G, "launches_per_step": G}
        if prof.get("valu_insts_per_launch"):
            roof["valu"] = valu_roofline(prof, kern_max)
            busy = roof["valu"].get("busy_frac")
            if pol is not None:  # rollout: the policy kernel (MFMA, the line's policy.roofline) holds most of the step
                roof["bound"] = "mfma"
                roof["bound_note"] = ("rollout step: the policy kernel (policy.roofline, MFMA) takes most of the step; "
                                      "achieved / peak / unit / frac are the env step's HBM figures over the whole step")
            elif busy is not None and busy > roof["frac"]:
                if busy >= 0.5:
                    roof["bound"] = "valu"
                    roof["bound_note"] = ("the SIMDs' VALU issue (roofline.valu.busy_frac, class-costed) is busier "
                                          "than HBM (frac); achieved / peak / unit / frac stay the HBM figures")
                else:  # config 2: one to three waves per SIMD, the serial path of a wave sets the step
                    roof["bound"] = "latency"
                    roof["bound_note"] = ("neither the VALU issue (roofline.valu.busy_frac) nor HBM (frac) is half "
                                          "busy: the launch is latency-bound; achieved / peak / unit / frac stay the "
                                          "HBM figures")
        metric = METRIC if pol is None else \
            "rollout agent-steps/sec (on-device policy + env step) at N=64 x E=8192 per MI355X"
        if tracker is not None:
            metric = metric.replace("agent-steps/sec", "eval-protocol agent-steps/sec (+ on-device eval metrics)", 1)
        if (n, e) != (64, 8192):  # a config line (--config / --drones / --envs), not the headline
            metric = metric.split(" at N=")[0] + f" at N={n} x E={e} envs per MI355X (not the headline shape)"
        rec = {
            "metric": metric, "value": value, "unit": "agent-steps/s", "n_gpus": world,
            "world_size": world_pg, "rank_devices": devs,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall_max / args.steps * 1e3,
            **({"ms_per_step_reps": [round(w / args.steps * 1e3, 6) for w in walls_rep]}
               if args.region_reps > 1 else {}),
            "ms_per_step_eager": eager_max / args.steps * 1e3, "step_timing": timing,
            "device_warmup": {"ms": round(warm_ms, 1), "steps": warm_steps,
                              "rehearsals": max(0, args.rehearse) if gatherer is None else 0,
                              "note": "untimed replays after the W warm-up steps, then untimed runs of the "
                                      "whole K-step region (rehearsals), before the timed region"},
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (device-RNG episodes, uniform(-1,1) actions)",
            "config": {"workload": f"N={n} drones x E={e} envs per GPU, "
                                   + ("kinematic dynamics + swarm reward" if args.dynamics == "kinematic"
                                      else "point-mass physics restatement (24 substeps) + physics reward")
                                   + ", in-kernel auto-reset"
                                   f"{', no-termination radii' if args.no_term else ''}"
                                   f"{', CTDE global_state emitted' if args.ctde else ''}",
                       "baseline_config": args.label,
                       "num_drones": n, "envs_per_gpu": e, "global_envs": world * e,
                       "obs_dim": vec.obs_dim,
                       "parallelism": f"env-sharded x{world}" + (f", {G} env groups per GPU on {G} HIP streams"
                                                                  if G > 1 else ""),
                       "ctde_allgather": gatherer is not None,
                       "ctde_gather_every": args.gather_every if gatherer is not None else None,
                       "ctde_gathers_timed": (sum(1 for k in gatherer.gathered_steps if k >= gather_t0)
                                              if gatherer is not None else None),
                       "ctde_gather_backend": gatherer.backend if gatherer is not None else None,
                       "dist_backend": dist.get_backend() if dist.is_initialized() else None},
            "roofline": roof,
            "env_done_fraction_last_step": done_frac,
            **({"rehearsal": f"{world} ranks sharing cuda:0 over gloo (SWARM_BENCH_REHEARSAL): the "
                             "multi-rank code path, not a scaling measurement"} if rehearsal else {}),
        }
        if pol is not None:
            rows = e * n
            flops = 2.0 * rows * (pol.in_dim * 256 + 256 * 256 + 256 * pol.out_dim)
            tf = flops / (pol_max * 1e-3) / 1e12
            rec["policy"] = {"precision": args.policy, "kernel": f"policy_mlp_{args.policy}",
                             "rows_per_launch": rows, "algorithmic_flops_per_launch": flops,
                             "kernel_ms_mean": pol_max,
                             "roofline": {"bound": "mfma", "achieved": tf,
                                          "peak": MFMA_PEAK_TFLOPS[args.policy], "unit": "TFLOP/s",
                                          "frac": tf / MFMA_PEAK_TFLOPS[args.policy]},
                             "weights": "random-init TorchFC [256, 256] relu (no checkpoint)"}
            rec["roofline"]["note"] = "env-step roofline fields cover the whole rollout step"
        if tracker is not None:
            rec["eval"] = {"tracker": ("EvalTracker fused into the step launches (swarm_step64_eval_once: episode "
                                       "reward, path length, exact formation error, votes, records)" if tracker.fused else
                                       "EvalTracker: swarm_eval_update per env group after its step (episode "
                                       "reward, path length, exact formation error, votes, records)"),
                           "fused": tracker.fused, "updates": tracker.updates}
        if not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline_port(n, e, args.cpu_seconds, raw, args.dynamics == "physics")
            if args.cpu_variant_seconds > 0 and not args.no_term and args.dynamics == "kinematic":
                rec["cpu_baseline_variants"] = cpu_python_variants(n, e, args.cpu_variant_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1 or own_pg:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- rank launcher
def _free_port() -> int:
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def check_world(gpus: int, env=None, device_count=None) -> tuple[int, str | None]:
    """(world, mode) for this process: mode "launch" = the parent spawns `gpus` ranks (WORLD_SIZE
    unset, --gpus > 1), None = run as this rank.  Raises SystemExit when the request cannot be met:
    WORLD_SIZE set and != --gpus, or fewer visible GPUs than ranks (one GPU per rank; the gloo
    rehearsal SWARM_BENCH_REHEARSAL=1 and the CPU stand-in SWARM_BENCH_STANDIN=cpu put every rank
    on one device / on the CPU and skip the device check)."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    shared = env.get("SWARM_BENCH_REHEARSAL") == "1" or env.get("SWARM_BENCH_STANDIN") == "cpu"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}: launch exactly --gpus ranks")
        mode = None
    else:
        world, mode = gpus, ("launch" if gpus > 1 else None)
    if not shared:
        if device_count is None:
            # the launcher parent never loads the HIP runtime (a child counts the devices; every
            # rank checks again before it touches its GPU, main()); a single rank counts itself
            device_count = count_devices_child() if mode == "launch" else _count_devices()
        if device_count < world:
            raise SystemExit(f"bench.py: --gpus {gpus} needs {world} GPUs (one rank per GPU), "
                             f"{device_count} visible")
    return world, mode


def _count_devices() -> int:
    import torch
    return torch.cuda.device_count()


def count_devices_child() -> int:
    """Visible GPUs, counted in a short-lived child process so that the launcher parent never
    imports torch or maps the HIP runtime before it starts the ranks."""
    p = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        raise SystemExit(f"bench.py: counting GPUs failed ({p.returncode}): {p.stderr[-500:]}")
    return int(p.stdout.strip().splitlines()[-1])


def launch_ranks(gpus: int, argv) -> int:
    """Parent of a multi-GPU run started as plain `python bench.py --gpus N`: spawn N fresh child
    processes (this file, same arguments) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set — before
    any GPU call here and without re-executing this process — forward rank 0's output, and return
    non-zero if any rank fails (the others are then stopped)."""
    import threading
    port = _free_port()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(gpus),
                LOCAL_WORLD_SIZE=str(gpus), GROUP_RANK="0", ROLE_RANK="0")
    cmd = [sys.executable, "-u", str(Path(__file__).resolve()), *argv]
    procs = []
    for r in range(gpus):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), ROLE_WORLD_SIZE=str(gpus))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    lines: list[str] = []

    def forward():  # rank 0's stdout, line by line, as it arrives
        for raw in procs[0].stdout:
            s = raw.decode(errors="replace")
            lines.append(s)
            sys.stdout.write(s)
            sys.stdout.flush()
    th = threading.Thread(target=forward, daemon=True)
    th.start()
    rc = 0
    live = set(range(gpus))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                sys.stderr.write(f"bench.py: rank {r} exited with {code}; stopping the other ranks\n")
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    th.join(timeout=10)
    if rc == 0:
        rec = [json.loads(s) for s in lines if s.startswith("{")]
        if not rec or rec[-1].get("n_gpus") != gpus:
            sys.stderr.write(f"bench.py: rank 0 reported no JSON line for {gpus} ranks\n")
            return 1
    return rc


def entry(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    world, mode = check_world(args.gpus)
    if mode == "launch":
        return launch_ranks(args.gpus, argv)
    if os.environ.get("SWARM_BENCH_STANDIN") == "cpu":
        standin_main(args)
        return 0
    main(argv)
    return 0


def standin_main(args) -> None:
    """SWARM_BENCH_STANDIN=cpu: the rank plumbing of main() (env-var ranks, gloo process group,
    shard plan, barrier-bracketed timed region, max over ranks, world size and per-rank devices in
    rank 0's line) with a CPU stand-in for the step, so tests can drive `python bench.py --gpus 2`
    without a GPU.  Not a measurement: `value` is the stand-in's rate and the line says so."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    if os.environ.get("SWARM_BENCH_STANDIN_FAIL_RANK") == str(rank):
        # tests: this rank fails while the others wait for it in the timed region's barrier
        raise SystemExit(f"stand-in rank {rank}: failing on request (SWARM_BENCH_STANDIN_FAIL_RANK)")
    offset, e = shard_plan(world, rank, args.envs)
    x = torch.zeros((e, args.drones, 3))
    # --ctde with several ranks: main()'s CTDE branch — a global_state slot ring written by every
    # step and all-gathered every --gather-every steps (distributed.GlobalStateGather over gloo)
    gatherer, gathers, ring, seen = None, set(), None, []
    if args.ctde and world > 1:
        from swarm_marl_amd.distributed import GlobalStateGather
        ring = torch.zeros((args.gs_slots, e, 6 * args.drones + 3))
        gatherer = GlobalStateGather(ring, lambda i: None, keep=2)
        gathers = set(gather_schedule(args.steps, args.gather_every))

    def step(k):
        x.add_(1.0)
        if gatherer is None:
            return
        s = gatherer.before_step()
        ring[s].fill_(float(1000 * rank + k))  # the step's global_state write-back
        gatherer.after_step(gather=k in gathers)
        if k in gathers:  # rank order of the concatenation (the values say which rank and step)
            out = gatherer.result()
            seen.append(bool(all(float(out[r * e, 0]) == 1000 * r + k for r in range(world))))

    def body():
        for k in range(args.steps):
            step(k)
    for k in range(args.warmup):
        x.add_(1.0)
    gather_t0 = gatherer.k if gatherer is not None else 0
    wall = timed_region(body, world, lambda: None)
    (wall_max,) = max_over_ranks([wall], world)
    devs = rank_devices(world, {"rank": rank, "device": "cpu", "env_offset": offset})
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": world * e * args.drones * args.steps / wall_max,
                          "unit": "agent-steps/s", "n_gpus": world, "world_size": world,
                          "rank_devices": devs, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": wall_max / args.steps * 1e3, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "standin": "CPU stand-in step (SWARM_BENCH_STANDIN=cpu): rank plumbing only, "
                                     "not a measurement",
                          "config": {"workload": f"N={args.drones} drones x E={e} envs per rank (stand-in)",
                                     "global_envs": world * e, "parallelism": f"env-sharded x{world}",
                                     "ctde_allgather": gatherer is not None,
                                     "ctde_gather_every": args.gather_every if gatherer is not None else None,
                                     "ctde_gathers_timed": (sum(1 for k in gatherer.gathered_steps if k >= gather_t0)
                                                            if gatherer is not None else None),
                                     "ctde_gather_backend": gatherer.backend if gatherer is not None else None,
                                     "ctde_rank_order_ok": all(seen) if gatherer is not None else None}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def rank_devices(world: int, mine: dict) -> list[dict]:
    """Every rank's device record (rank order), gathered outside the timed region."""
    if world == 1:
        return [mine]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


if __name__ == "__main__":
    sys.exit(entry())
