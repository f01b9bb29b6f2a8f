"""Fixed cost of a timed region: wall and event time of K-step regions for K = 1 .. 40.

    python tools/k20_intercept.py [groups] [reps]

Launches as bench.py's eager short region (VecSwarm.step_groups, one native call per step).
Two bracket styles per K: 'fork' (bench.py: a start event on group stream 0 that the other
streams wait for, joins and an end event on stream 0) and 'free' (a start and an end event on
every group stream, no waits; the device sync alone closes the region).  Prints the median wall
and event us per region and the least-squares intercept / slope over K.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multi-agent-rl-for-autonomous-drone-swarms_amd"))
from swarm_marl_amd import VecSwarm  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
dev = torch.device("cuda", 0)
vec = VecSwarm(8192, {"num_drones": 64}, device=dev, auto_reset=True, seed=0, groups=G)
vec.reset()
gen = torch.Generator(device=dev).manual_seed(1000)
ring = [torch.rand((8192, 64, 3), device=dev, generator=gen) * 2 - 1 for _ in range(8)]
sts = vec.group_streams
s0 = sts[0]
torch.cuda.synchronize()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for k in range(64):
        vec.step_groups(ring[k % 8])
    torch.cuda.synchronize()


def region(K, style):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in sts]
    torch.cuda.synchronize()
    a = time.perf_counter()
    if style == "fork":
        evs[0][0].record(s0)
        for st in sts[1:]:
            st.wait_event(evs[0][0])
    else:
        for (e0, _), st in zip(evs, sts):
            e0.record(st)
    for k in range(K):
        vec.step_groups(ring[k % 8])
    if style == "fork":
        for st in sts[1:]:
            s0.wait_stream(st)
        evs[0][1].record(s0)
    else:
        for (_, e1), st in zip(evs, sts):
            e1.record(st)
    torch.cuda.synchronize()
    w = (time.perf_counter() - a) * 1e6
    if style == "fork":
        ev = evs[0][0].elapsed_time(evs[0][1]) * 1e3
    else:
        first = evs[0][0]
        ev = max(first.elapsed_time(e1) for _, e1 in evs) * 1e3 - min(first.elapsed_time(e0) for e0, _ in evs) * 1e3
    return w, ev


Ks = [1, 2, 3, 5, 10, 20, 40]
res = {}
for r in range(reps):
    for style in ("fork", "free"):
        for K in Ks:
            res.setdefault((style, K), []).append(region(K, style))
empty = []
for _ in range(10):
    torch.cuda.synchronize()
    a = time.perf_counter()
    torch.cuda.synchronize()
    empty.append((time.perf_counter() - a) * 1e6)
print(f"groups={G}  idle sync {np.median(empty):.1f} us")
for style in ("fork", "free"):
    xs, ws, es = [], [], []
    for K in Ks:
        v = np.array(res[(style, K)])
        w, e = np.median(v[:, 0]), np.median(v[:, 1])
        xs.append(K); ws.append(w); es.append(e)
        print(f"{style} K={K:3d}: wall {w:7.1f} us ({w / K:5.1f}/step)  events {e:7.1f} us ({e / K:5.1f}/step)")
    bw = np.polyfit(xs, ws, 1)
    be = np.polyfit(xs, es, 1)
    print(f"{style}: wall = {bw[1]:.1f} + {bw[0]:.2f} K   events = {be[1]:.1f} + {be[0]:.2f} K")
