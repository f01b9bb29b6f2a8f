"""On-device eval metric cost: ms per step of VecSwarm.step alone vs step + EvalTracker.update
(one swarm_eval_update launch) at N drones x E envs, and the finished-episode count.
    python tools/eval_bench.py [E] [N] [steps]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import torch

from swarm_marl_amd import VecSwarm
from swarm_marl_amd.eval_metrics import EvalTracker

E = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
dev = torch.device("cuda", 0)
vec = VecSwarm(E, {"num_drones": N}, device=dev, auto_reset=True, seed=0, with_infos=True)
vec.reset()
ev = EvalTracker(vec, capacity=1 << 21, fused=False)  # the unfused update kernel, as documented
ev.begin()
g = torch.Generator(device=dev).manual_seed(1)
ring = [torch.rand((E, N, 3), device=dev, generator=g) * 2 - 1 for _ in range(8)]
res = {}
for mode in ("step", "step+eval", "step", "step+eval"):
    for k in range(20):
        vec.step(ring[k % 8])
        if mode == "step+eval":
            ev.update()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for k in range(K):
        vec.step(ring[k % 8])
        if mode == "step+eval":
            ev.update()
    b.record()
    torch.cuda.synchronize()
    res[mode] = a.elapsed_time(b) / K
print(json.dumps({"E": E, "N": N, "ms_per_step": res["step"], "ms_per_step_with_eval": res["step+eval"],
                  "eval_ms_per_step": res["step+eval"] - res["step"], "episodes_recorded": int(ev.count.sum()),
                  "aggregate": ev.aggregate()}))
