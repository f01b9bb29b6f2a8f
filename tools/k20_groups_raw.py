"""Driver-length (K = 20) timed regions with 2 / 3 / 4 env groups: launches through
`with torch.cuda.stream(st): vec.step_group(...)` (bench.py's eager loop) against raw-handle
launches (`vec._launch_step` with the group stream handles, no stream context per launch).

    python tools/k20_groups_raw.py [reps]

Per (groups, launch mode) and rep: wall us per step of the bracketed region (sync .. launches ..
sync), the host's enqueue time per step, and the bracket events' time per step.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multi-agent-rl-for-autonomous-drone-swarms_amd"))
from swarm_marl_amd import VecSwarm  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
K = 20
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(1000)
ring = [torch.rand((8192, 64, 3), device=dev, generator=gen) * 2 - 1 for _ in range(8)]
res = {}
vecs = {}
for G in (2, 3, 4):
    vec = VecSwarm(8192, {"num_drones": 64}, device=dev, auto_reset=True, seed=0, groups=G)
    vec.reset()
    vecs[G] = vec
torch.cuda.synchronize()


def run(G, mode, steps):
    vec = vecs[G]
    sts = vec.group_streams
    hs = vec._gstream_h
    s0 = sts[0]
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    torch.cuda.synchronize()
    a = time.perf_counter()
    ev[0].record(s0)
    for st in sts[1:]:
        st.wait_event(ev[0])
    for k in range(steps):
        act = ring[k % 8]
        if mode == "ctx":
            for g, st in enumerate(sts):
                with torch.cuda.stream(st):
                    vec.step_group(g, act)
        else:
            for g in range(G):
                vec._launch_step(g, act, None, hs[g])
    for st in sts[1:]:
        s0.wait_stream(st)
    ev[1].record(s0)
    b = time.perf_counter()
    torch.cuda.synchronize()
    c = time.perf_counter()
    return (c - a) / steps * 1e6, (b - a) / steps * 1e6, ev[0].elapsed_time(ev[1]) / steps * 1e3


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.4:  # clocks up
    for G in (2, 3, 4):
        run(G, "raw", 40)
for r in range(reps):
    for G in (2, 3, 4):
        for mode in ("ctx", "raw"):
            for _ in range(3):  # warm this configuration's queues
                run(G, mode, 8)
            res.setdefault((G, mode), []).append(run(G, mode, K))
for (G, mode), v in sorted(res.items()):
    v = np.array(v)
    print(f"groups={G} {mode:3s} K={K}: wall {np.median(v[:, 0]):5.1f} us/step [{v[:, 0].min():.1f}-{v[:, 0].max():.1f}]  "
          f"host {np.median(v[:, 1]):4.1f}  events {np.median(v[:, 2]):5.1f} [{v[:, 2].min():.1f}-{v[:, 2].max():.1f}]")
for G in (2, 3, 4):
    for mode in ("ctx", "raw"):
        v = np.array([run(G, mode, 400) for _ in range(3)])
        print(f"groups={G} {mode:3s} K=400: wall {np.median(v[:, 0]):5.1f} us/step  host {np.median(v[:, 1]):4.1f}  "
              f"events {np.median(v[:, 2]):5.1f}")
