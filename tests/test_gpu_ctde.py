"""GPU: the CTDE global_state all-gather of bench.py (BASELINE config 5), overlapped.

Reference contract: the critic input is the per-step global_state (drone_swarm_env.py:293-302)
collected for every step of a batch (training/callbacks.py:14-57; global_state_dim = 6N+3,
config_builders.py:164).  bench.py --ctde gathers it every `--gather-every` steps with
distributed.GlobalStateGather: the step writes slot k % R of a device ring and the gather runs
over RCCL on a side stream while the next steps run on the two env-group streams.  Here a
one-rank RCCL process group drives that exact path and the gathered tensors must equal, bit for
bit, a synchronous join-then-gather of a single-stream, single-buffer run of the same batch.
"""
from __future__ import annotations

import json
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def pg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        yield torch.device("cuda", 0)
    finally:
        dist.destroy_process_group()


def _acts(dev, e, n, k):
    g = torch.Generator(device=dev).manual_seed(900 + k)
    return torch.rand((e, n, 3), device=dev, generator=g) * 2 - 1


@pytest.mark.parametrize("e,n,groups,slots,every", [(512, 64, 2, 4, 2), (96, 256, 2, 3, 1), (300, 16, 3, 2, 3)])
def test_overlapped_gather_equals_synchronous(pg, e, n, groups, slots, every):
    import bench
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.distributed import GlobalStateGather, gather_global_state
    dev = pg
    steps = 11
    sched = set(bench.gather_schedule(steps, every))
    kw = dict(device=dev, auto_reset=True, seed=21, with_global_state=True)
    # the bench's path: env groups on their streams, slot ring, side-stream RCCL gather, no joins
    a = VecSwarm(e, {"num_drones": n}, groups=groups, global_state_slots=slots, **kw)
    # reference: one launch per step on the current stream, one buffer, join + gather inline
    b = VecSwarm(e, {"num_drones": n}, **kw)
    a.reset()
    b.reset()
    g = GlobalStateGather(a.global_state_ring, a.select_global_state_slot, keep=len(sched))
    assert g.world == 1 and g.backend == "nccl" and not g.staged
    acts = [_acts(dev, e, n, k) for k in range(steps)]
    for st in a.group_streams:  # the group streams start after the reset and the action draws
        st.wait_stream(torch.cuda.current_stream(dev))
    ref = {}
    for k in range(steps):
        g.before_step(a.group_streams)
        for gi, st in enumerate(a.group_streams):
            with torch.cuda.stream(st):
                a.step_group(gi, acts[k])
        g.after_step(a.group_streams, gather=k in sched)
        b.step(acts[k])
        if k in sched:
            ref[k] = gather_global_state(b.global_state).clone()
    a.join()
    g.wait()
    torch.cuda.synchronize()
    assert g.gathered_steps == sorted(sched)
    for i, k in enumerate(g.gathered_steps):
        assert torch.equal(g.result(i), ref[k]), f"gather at step {k}"
        # the slot that step k wrote still holds it unless a later step reused the slot
        if k + slots >= steps:
            assert torch.equal(a.global_state_ring[k % slots], ref[k])
    assert torch.equal(a.obs, b.obs) and torch.equal(a.pos, b.pos)


@pytest.mark.parametrize("groups", [2, 4])
def test_graph_segment_gather_equals_synchronous(pg, groups):
    """bench.py's graph-replayed gathering run: per group, two hipGraphs of `ring` steps, each with
    its global_state slots (one half of a 2 x ring ring) baked in at capture; a segment replay is
    followed by the gather of its last slot (GlobalStateGather.before_steps / after_step), which
    overlaps the next segment.  Every gather equals a synchronous run's, bit for bit."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.distributed import GlobalStateGather, gather_global_state
    dev = pg
    e, n, ring, segs = 512, 64, 4, 7
    kw = dict(device=dev, auto_reset=True, seed=33, with_global_state=True)
    a = VecSwarm(e, {"num_drones": n}, groups=groups, global_state_slots=2 * ring, **kw)
    b = VecSwarm(e, {"num_drones": n}, **kw)
    a.reset()
    b.reset()
    acts = [_acts(dev, e, n, 700 + k) for k in range(ring)]
    torch.cuda.synchronize()
    halves = []
    for h in range(2):
        gs = []
        for gi, st in enumerate(a.group_streams):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.stream(st), torch.cuda.graph(gr, stream=st, capture_error_mode="thread_local"):
                for k in range(h * ring, (h + 1) * ring):
                    a.select_global_state_slot(k % (2 * ring))
                    a.step_group(gi, acts[k % ring])
            gs.append(gr)
        halves.append(gs)
    torch.cuda.synchronize()  # capture runs nothing: a and b are still at the same reset state
    g = GlobalStateGather(a.global_state_ring, a.select_global_state_slot, keep=segs)
    start = torch.cuda.Event()
    start.record(torch.cuda.current_stream(dev))
    for st in a.group_streams:
        st.wait_event(start)
    ref = []
    for j in range(segs):
        g.before_steps(ring, a.group_streams)
        for gi, st in enumerate(a.group_streams):
            with torch.cuda.stream(st):
                halves[(g.k // ring) % 2][gi].replay()
        for i in range(ring):
            g.after_step(a.group_streams, gather=i == ring - 1)
        for i in range(ring):
            b.step(acts[i])
        ref.append(gather_global_state(b.global_state).clone())
    a.join()
    g.wait()
    torch.cuda.synchronize()
    assert g.gathered_steps == [ring * j + ring - 1 for j in range(segs)]
    for j in range(segs):
        assert torch.equal(g.result(j), ref[j]), f"gather after segment {j}"
    assert torch.equal(a.obs, b.obs) and torch.equal(a.pos, b.pos)


def test_bench_ctde_graph_gather_line_one_rank(pg, capsys):
    """bench.main's graph-replayed gathering run (--graph-gather, K > 256, --gather-every = --ring): the line
    reports graph replay, 2 x ring slots and every scheduled gather inside the timed region."""
    import bench
    bench_args = ["--config", "n256", "--envs", "64", "--steps", "260", "--warmup", "3", "--graph-gather",
                  "--device-warmup-ms", "1", "--no-cpu-baseline", "--cpu-variant-seconds", "0"]
    rec = _run_main_with_world(bench, bench_args, capsys)
    cfg = rec["config"]
    assert cfg["ctde_allgather"] is True and cfg["ctde_gather_every"] == 8
    assert cfg["ctde_gathers_timed"] == len(bench.gather_schedule(260, 8))
    assert "hipGraph replay" in rec["step_timing"] and "16-slot ring" in rec["step_timing"]
    assert rec["value"] > 0


@pytest.mark.parametrize("mode", ["auto", "new"])
def test_result_buffers_reused_after_consumer_reads(pg, mode):
    """keep=1 < gathers: every gather overwrites the previous one's buffer.  The consumer queues
    a copy of each result on the current stream right after wait() (no host sync); the gather
    that reuses the buffer must order after that copy (consumer-stream event)."""
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.distributed import GlobalStateGather, gather_global_state
    dev = pg
    e, n, steps = 256, 64, 9
    kw = dict(device=dev, auto_reset=True, seed=5, with_global_state=True)
    a = VecSwarm(e, {"num_drones": n}, groups=2, global_state_slots=2, **kw)
    b = VecSwarm(e, {"num_drones": n}, **kw)
    a.reset()
    b.reset()
    g = GlobalStateGather(a.global_state_ring, a.select_global_state_slot, keep=1, stream=mode)
    acts = [_acts(dev, e, n, 50 + k) for k in range(steps)]
    for st in a.group_streams:
        st.wait_stream(torch.cuda.current_stream(dev))
    got, ref = [], []
    for k in range(steps):
        g.before_step(a.group_streams)
        for gi, st in enumerate(a.group_streams):
            with torch.cuda.stream(st):
                a.step_group(gi, acts[k])
        g.after_step(a.group_streams, gather=True)
        g.wait()
        got.append(g.result().clone())  # queued on the current stream, read before the reuse
        b.step(acts[k])
        ref.append(gather_global_state(b.global_state).clone())
    if mode == "auto":  # two env groups: the gathers go out from the default stream
        assert g.stream == torch.cuda.default_stream(dev)
    else:
        assert g.stream != torch.cuda.default_stream(dev)
    torch.cuda.synchronize()
    for k in range(steps):
        assert torch.equal(got[k], ref[k]), f"gather {k}"


def test_bench_ctde_rehearsal_line_one_rank(pg, capsys):
    """bench.main's CTDE branch end to end on one rank (RCCL group of one): the gather runs every
    --gather-every steps inside the timed region and the line says so."""
    import bench
    bench_args = ["--config", "n256", "--envs", "64", "--steps", "16", "--warmup", "2",
                  "--device-warmup-ms", "0", "--no-cpu-baseline", "--gather-every", "4"]
    # main() gathers only with several ranks unless SWARM_BENCH_FORCE_GATHER=1 (one-rank RCCL group)
    import torch.distributed as dist
    assert dist.is_initialized()
    rec = _run_main_with_world(bench, bench_args, capsys)
    cfg = rec["config"]
    assert cfg["ctde_allgather"] is True and cfg["ctde_gather_every"] == 4
    assert cfg["ctde_gathers_timed"] == 4 and cfg["ctde_gather_backend"] == "nccl"
    assert rec["value"] > 0


def _run_main_with_world(bench, argv, capsys):
    old = os.environ.get("SWARM_BENCH_FORCE_GATHER")
    os.environ["SWARM_BENCH_FORCE_GATHER"] = "1"
    try:
        bench.main(argv)
    finally:
        if old is None:
            os.environ.pop("SWARM_BENCH_FORCE_GATHER", None)
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)
