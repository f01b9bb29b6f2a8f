"""Dict-API latency: agent-steps/s of DroneSwarmEnv (E = 1, the RLlib MultiAgentEnv surface the
reference's train_*.py use) with uniform(-1,1) actions and reset on __all__, agent-steps counted
as len(rewards) like BASELINE.md §3 (reference: 10,825 / 6,277 agent-steps/s per core at N=4/16).
    python tools/dict_bench.py [seconds] [N ...]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import numpy as np

from swarm_marl_amd.envs import DroneSwarmEnv

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
ns = [int(x) for x in sys.argv[2:]] or [3, 4, 16]
REF = {4: 10825, 16: 6277, 64: 1726}
for n in ns:
    env = DroneSwarmEnv({"num_drones": n, "seed": 0})
    rng = np.random.default_rng(1)
    obs, _ = env.reset(seed=0)
    for _ in range(50):  # warm-up
        acts = {a: rng.uniform(-1, 1, 3).astype(np.float32) for a in obs}
        obs, rew, term, trunc, _ = env.step(acts)
        if term["__all__"] or trunc["__all__"]:
            obs, _ = env.reset()
    steps = agent_steps = resets = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        acts = {a: rng.uniform(-1, 1, 3).astype(np.float32) for a in obs}
        obs, rew, term, trunc, _ = env.step(acts)
        steps += 1
        agent_steps += len(rew)
        if term["__all__"] or trunc["__all__"]:
            obs, _ = env.reset()
            resets += 1
    el = time.perf_counter() - t0
    print(json.dumps({"N": n, "env_steps_per_s": steps / el, "agent_steps_per_s": agent_steps / el,
                      "us_per_step": el / steps * 1e6, "resets": resets,
                      "reference_agent_steps_per_s_per_core": REF.get(n)}), flush=True)
