"""Per-wave lifetimes of swarm_step16q over many steps, with the slow paths each wave took
(diagnostic; a full -DSWARM_STAMPS build, e.g. tools/variants_fast.sh with -DSWARM_STAMPS):
    SWARM_STAMPS_LIB=build/var/stamps16.so python tools/stamps16.py [E] [steps]
Flags: 1 / 16 quad exact-selection finish of the neighbours / obstacles (near-tie or unproven bound),
2 exact pair-collision band, 4 reset, 8 masked pass."""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ["SWARM_MI355X_LIB"] = os.environ.get("SWARM_STAMPS_LIB", str(ROOT / "build" / "var" / "stamps16.so"))
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from swarm_marl_amd import VecSwarm  # noqa: E402
from swarm_marl_amd import _native as nat  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
K = int(sys.argv[2]) if len(sys.argv) > 2 else 60
vec = VecSwarm(E, {"num_drones": 16}, device="cuda:0", auto_reset=True, seed=0)
vec.reset()
lib = nat.load_library()
lib.swarm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
g = torch.Generator(device="cuda:0").manual_seed(1)
acts = [torch.rand((E, 16, 3), device="cuda:0", generator=g) * 2 - 1 for _ in range(8)]
buf = np.zeros(E * 16, np.uint64)
rows = []
for k in range(K):
    vec.step(acts[k % 8])
    torch.cuda.synchronize()
    lib.swarm_debug_stamps(buf.ctypes.data, buf.size)
    st = buf.reshape(E, 16).astype(np.int64)
    life = (st[:, 12] - st[:, 11]) / 100.0
    start = (st[:, 11] - st[:, 11].min()) / 100.0
    rows.append((life, st[:, 13] & 31, start, np.diff(st[:, 0:9], axis=1)))
life = np.stack([r[0] for r in rows[5:]])
flags = np.stack([r[1] for r in rows[5:]])
print(f"E={E}: per-step max wave life us: median {np.median(life.max(1)):.2f}  p90 {np.percentile(life.max(1), 90):.2f}; "
      f"median wave {np.median(life):.2f}")
for f in range(32):
    m = flags == f
    if m.any():
        print(f"  flags {f:2d}: waves/step {m.sum() / len(life):7.2f}  life median {np.median(life[m]):.2f}  max {life[m].max():.2f}")
am = life.argmax(1)
print("slowest wave per step (flags):", [int(flags[i, am[i]]) for i in range(min(20, len(am)))])
PHASES = ["w0load", "w0integ", "w0pass", "w0reward+writes", "w1pass-w0end", "w1finish", "w1stage", "w1wait+store"]
ph = np.concatenate([r[3] for r in rows[5:]])
fl = flags.reshape(-1)
for f in sorted(set(fl.tolist())):
    m = fl == f
    if m.sum() >= 5:
        print(f"  phase cycles (median) flags {f:2d}: " +
              " ".join(f"{n} {int(np.median(ph[m, i]))}" for i, n in enumerate(PHASES)))
