"""How often the headline step takes step64's general finish (diagnostic; a stamps build with
-DSWARM_DIAG_FINISH):
    python tools/stamps.py build -DSWARM_DIAG_FINISH      (-> build/stamps/libswarm_stamps.so)
    SWARM_MI355X_LIB=<that .so> python tools/finish_diag.py [steps]
Counters: select_topk calls (waves), waves / lanes failing the straight-line finish, waves / lanes
needing exact_select (neighbours, obstacles), general finishes after a reset (s' keys)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multi-agent-rl-for-autonomous-drone-swarms_amd"))
from swarm_marl_amd import VecSwarm  # noqa: E402
from swarm_marl_amd import _native as nat  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 60
vec = VecSwarm(8192, {"num_drones": 64}, device="cuda:0", auto_reset=True, seed=0)
vec.reset()
gen = torch.Generator(device="cuda:0").manual_seed(1000)
ring = [torch.rand((8192, 64, 3), device="cuda:0", generator=gen) * 2 - 1 for _ in range(8)]
lib = nat.load_library()
lib.swarm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
n = (1 << 19) + 8
buf = np.zeros(n, np.uint64)
for k in range(K):
    vec.step(ring[k % 8])
torch.cuda.synchronize()
assert lib.swarm_debug_stamps(buf.ctypes.data, n) == 0
c = buf[1 << 19:].astype(float)
print(f"steps {K}: select_topk waves {c[0]:.0f}; general finish: waves {c[1] / c[0]:.4f}, lanes {c[2] / c[0] / 64:.5f}; "
      f"exact_select nb: waves {c[3] / c[0]:.4f}, lanes {c[4] / c[0] / 64:.5f}; ob: waves {c[5] / c[0]:.4f}, "
      f"lanes {c[6] / c[0] / 64:.5f}; general after reset {c[7] / max(c[1], 1):.3f} of general")
