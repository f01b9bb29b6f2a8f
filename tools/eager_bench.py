"""Host cost of eager VecSwarm launches (no hipGraph): µs of Python per call and the eager
whole-step rate, for the headline shape (1 and 2 env groups), config 2 and a dict-API-sized batch.

    python tools/eager_bench.py
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import torch  # noqa: E402
from swarm_marl_amd import VecSwarm  # noqa: E402

dev = torch.device("cuda", 0)
for e, n, g in ((8192, 64, 1), (8192, 64, 2), (1024, 16, 1), (1, 4, 1)):
    vec = VecSwarm(e, {"num_drones": n}, device=dev, auto_reset=True, seed=0, groups=g)
    vec.reset()
    acts = [torch.rand((e, n, 3), device=dev) * 2 - 1 for _ in range(8)]
    for k in range(50):
        vec.step(acts[k % 8])
    torch.cuda.synchronize()
    # host time per call: launches only (the GPU queue absorbs them)
    K = 200
    t0 = time.perf_counter()
    for k in range(K):
        vec.step(acts[k % 8])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"E={e} N={n} groups={g}: host {1e6 * (t1 - t0) / K:6.2f} us per step() call, "
          f"eager wall {1e6 * (t2 - t0) / K:6.2f} us per step", flush=True)
