"""Diagnostic: which HIP streams make env groups overlap.  Each spec builds VecSwarm(groups=G),
optionally replaces its group streams (hi = high-priority pool, raw = hipStreamCreate via ctypes),
and times 400 graph-replayed steps bracketed on group stream 0.
    python tools/groups_exp3.py G:kind ..."""
import ctypes
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import torch
from swarm_marl_amd import VecSwarm

dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
E, N, RING, REPS = 8192, 64, 8, 50
for spec in sys.argv[1:]:
    G, kind = spec.split(":")
    G = int(G)
    vec = VecSwarm(E, {"num_drones": N}, device=dev, auto_reset=True, seed=0, groups=G)
    if kind == "hi":
        vec.group_streams = [torch.cuda.Stream(dev, priority=-1) for _ in range(G)]
    elif kind == "raw":
        sts = []
        for _ in range(G):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0
            sts.append(torch.cuda.ExternalStream(h.value, device=dev))
        vec.group_streams = sts
    vec.reset()
    gen = torch.Generator(device=dev).manual_seed(1000)
    ring = [torch.rand((E, N, 3), device=dev, generator=gen) * 2 - 1 for _ in range(RING)]
    sts = vec.group_streams
    torch.cuda.synchronize()
    # eager pass
    bs = sts[0]
    for mode in ("eager", "graph"):
        if mode == "graph":
            graphs = []
            for g, st in enumerate(sts):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.stream(st), torch.cuda.graph(gr, stream=st):
                    for k in range(RING):
                        vec.step_group(g, ring[k])
                graphs.append(gr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(bs)
        for st in sts[1:]:
            st.wait_event(e0)
        for r in range(REPS):
            for g, st in enumerate(sts):
                with torch.cuda.stream(st):
                    if mode == "graph":
                        graphs[g].replay()
                    else:
                        for k in range(RING):
                            vec.step_group(g, ring[k])
        for st in sts[1:]:
            bs.wait_stream(st)
        e1.record(bs)
        torch.cuda.synchronize()
        print(f"{spec} {mode}: {e0.elapsed_time(e1) / (REPS * RING) * 1e3:.2f} us/step", flush=True)
    del vec, ring, graphs
    torch.cuda.synchronize()
