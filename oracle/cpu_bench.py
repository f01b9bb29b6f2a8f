"""One CPU-baseline worker process (TEST INFRASTRUCTURE / bench.py cpu_baseline leg only).

    python -m oracle.cpu_bench --kind loop|numpy --drones N --envs E --seconds S --seed K

Prints one JSON line {"agent_steps": ..., "seconds": ...}.  bench.py starts one such process
per host core (one process per core, E split across them), each single-threaded.
  loop  : oracle/swarm_loop.py, per-agent loops like the reference DroneSwarmEnv.step
  numpy : oracle/swarm_oracle.py, vectorised over the process's envs (auto-reset on)
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np


def run_numpy(n: int, e: int, seconds: float, seed: int) -> tuple[int, float]:
    from oracle import swarm_oracle as so
    cfg = so.make_cfg(num_drones=n)
    st, _ = so.reset_device(cfg, so.empty_state(cfg, e), seed=seed, env_offset=seed * e)
    rng = np.random.default_rng(1000 + seed)
    ring = [rng.uniform(-1, 1, (e, n, 3)).astype(np.float32) for _ in range(4)]
    st, _ = so.step(cfg, st, ring[0], auto_reset=True, seed=seed, env_offset=seed * e)  # warm
    count, k, t0 = 0, 0, time.perf_counter()
    while True:
        st, _ = so.step(cfg, st, ring[k % 4], auto_reset=True, seed=seed, env_offset=seed * e)
        count += e * n
        k += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return count, el


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=("loop", "numpy"), required=True)
    ap.add_argument("--drones", type=int, required=True)
    ap.add_argument("--envs", type=int, required=True)
    ap.add_argument("--seconds", type=float, required=True)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    if a.kind == "loop":
        from oracle.swarm_loop import run_for
        count, el = run_for(a.envs, a.drones, a.seconds, seed=a.seed)
    else:
        count, el = run_numpy(a.drones, a.envs, a.seconds, a.seed)
    print(json.dumps({"agent_steps": count, "seconds": el}), flush=True)


if __name__ == "__main__":
    main()
