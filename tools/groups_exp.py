"""Diagnostic: E envs per GPU as G independent env groups (E/G envs each, env_offset g*E/G), each
stepped on its own HIP stream from its own hipGraph of ring steps.  Prints ms per whole-batch step.
    python tools/groups_exp.py [E] [G...]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import torch
from swarm_marl_amd import VecSwarm

E = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
GS = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 1, 2, 4]
dev = torch.device("cuda", 0)
RING, REPS, N = 8, 60, 64
for G in GS:
    eg = E // G
    vecs = [VecSwarm(eg, {"num_drones": N}, device=dev, auto_reset=True, seed=0, env_offset=g * eg)
            for g in range(G)]
    for v in vecs:
        v.reset()
    gen = torch.Generator(device=dev).manual_seed(1000)
    rings = [[torch.rand((eg, N, 3), device=dev, generator=gen) * 2 - 1 for _ in range(RING)] for _ in range(G)]
    streams = [torch.cuda.Stream(dev) for _ in range(G)]
    torch.cuda.synchronize()
    graphs = []
    for g in range(G):
        for k in range(20):
            vecs[g].step(rings[g][k % RING])
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(streams[g]):
            with torch.cuda.graph(gr, stream=streams[g]):
                for k in range(RING):
                    vecs[g].step(rings[g][k])
        graphs.append(gr)
    torch.cuda.synchronize()
    for g in range(G):
        with torch.cuda.stream(streams[g]):
            graphs[g].replay()
    torch.cuda.synchronize()
    main = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(main)
    for s in streams:
        s.wait_event(e0)
    for _ in range(REPS):
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                graphs[g].replay()
    for s in streams:
        ev = torch.cuda.Event()
        ev.record(s)
        main.wait_event(ev)
    e1.record(main)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = REPS * RING
    print(f"E={E} G={G}: events {e0.elapsed_time(e1) / steps * 1e3:.2f} us/step, wall {wall / steps * 1e6:.2f} us/step, "
          f"{E * N * steps / wall:.3e} agent-steps/s", flush=True)
    del graphs, vecs, rings
    torch.cuda.synchronize()
