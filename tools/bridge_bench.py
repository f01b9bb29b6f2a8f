"""RLlib bridge throughput: agent-steps/s of SwarmBaseEnv (poll + send_actions of MultiEnvDicts,
one launch for all E envs) with uniform(-1,1) actions built per agent, try_reset on __all__.
    python tools/bridge_bench.py [seconds] E:N ..."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import numpy as np

from swarm_marl_amd.rllib_bridge import SwarmBaseEnv

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
for spec in sys.argv[2:] or ["256:4", "1024:4", "64:64"]:
    e, n = (int(x) for x in spec.split(":"))
    for mode in ("info", "device"):
        br = SwarmBaseEnv(e, {"num_drones": n}, seed=0, global_state=mode)
        rng = np.random.default_rng(0)
        obs = br.poll()[0]
        steps = agent_steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            br.send_actions({i: {a: rng.uniform(-1, 1, 3).astype(np.float32) for a in o} for i, o in obs.items()})
            obs, rew, term, trunc, infos, _ = br.poll()
            steps += 1
            agent_steps += sum(len(r) for r in rew.values())
            for i, t in term.items():
                if t["__all__"] or trunc[i]["__all__"]:
                    o2, _ = br.try_reset(i)
                    obs[i] = o2[i]
        el = time.perf_counter() - t0
        print(json.dumps({"E": e, "N": n, "global_state": mode, "agent_steps_per_s": agent_steps / el,
                          "ms_per_step": el / steps * 1e3}), flush=True)
