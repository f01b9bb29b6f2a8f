"""Per-wave timeline of the headline step with env groups (diagnostic; a -DSWARM_STAMPS build).

Build:  python tools/stamps.py build            -> build/stamps/libswarm_stamps.so
Run:    SWARM_STAMPS_LIB=build/stamps/libswarm_stamps.so python tools/stamps_groups.py [groups] [steps] [stagger_us]

After `steps` eager steps (group g on its own stream) the stamps hold every env's LAST step:
wave start / end (s_memrealtime, 100 MHz, chip-wide) and the phase boundaries (s_memtime,
mapped to real time per wave).  Prints, per group and per 1-us bin, how many waves are in their
compute phase (start .. obs row build) and in their obs store phase (.. end): the overlap of one
group's stores with the other's compute is what env groups are for.
"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LIB = Path(os.environ.get("SWARM_STAMPS_LIB", ROOT / "build" / "stamps" / "libswarm_stamps.so"))
os.environ["SWARM_MI355X_LIB"] = str(LIB)
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from swarm_marl_amd import VecSwarm  # noqa: E402
from swarm_marl_amd import _native as nat  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
stagger_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
E, N = 8192, 64
vec = VecSwarm(E, {"num_drones": N}, device="cuda:0", auto_reset=True, seed=0, groups=G)
vec.reset()
gen = torch.Generator(device="cuda:0").manual_seed(1)
acts = [torch.rand((E, N, 3), device="cuda:0", generator=gen) * 2 - 1 for _ in range(8)]
torch.cuda.synchronize()
streams = vec.group_streams or [torch.cuda.current_stream()]
if stagger_us > 0 and G > 1:
    with torch.cuda.stream(streams[1]):
        torch.cuda._sleep(int(stagger_us * 2400))
for k in range(K):
    for g, st in enumerate(streams):
        with torch.cuda.stream(st):
            vec.step_group(g, acts[k % 8])
torch.cuda.synchronize()
lib = nat.load_library()
lib.swarm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(E * 16, np.uint64)
assert lib.swarm_debug_stamps(buf.ctypes.data, buf.size) == 0
st = buf.reshape(E, 16).astype(np.int64)
mt, rt0, rt1 = st[:, :9], st[:, 11], st[:, 12]
scale = (rt1 - rt0) / np.maximum(mt[:, 8] - mt[:, 0], 1)  # realtime ticks per shader cycle, per wave
rt = rt0[:, None] + (mt - mt[:, :1]) * scale[:, None]      # phase boundaries in realtime ticks
t0 = rt0.min()
us = lambda x: (x - t0) / 100.0  # noqa: E731  (100 MHz)
reset = (vec.env_done.cpu().numpy() & 4) != 0
print(f"groups={G} steps={K} stagger={stagger_us}us  clock {1 / np.median(scale) / 100:.2f} GHz  "
      f"resets {reset.mean():.3f}")
for g, (lo, hi) in enumerate(vec.group_slices):
    s = slice(lo, hi)
    print(f"group {g}: start {np.percentile(us(rt0[s]), [0, 50, 100]).round(2)}  "
          f"obs-phase {np.percentile(us(rt[s, 7]), [0, 50, 100]).round(2)}  end {np.percentile(us(rt1[s]), [0, 50, 100]).round(2)} us")
    ph = np.diff(mt[s], axis=1)
    print("   phase cycles (median): " + " ".join(f"{x:.0f}" for x in np.median(ph, axis=0)))
span = us(rt1.max())
bins = np.arange(0, span + 1.0, 1.0)
print("  t(us) " + "  ".join(f"g{g}:comp/store" for g in range(G)))
for b in bins:
    row = []
    for g, (lo, hi) in enumerate(vec.group_slices):
        s = slice(lo, hi)
        comp = np.sum((us(rt0[s]) <= b + 0.5) & (us(rt[s, 7]) > b + 0.5))
        sto = np.sum((us(rt[s, 7]) <= b + 0.5) & (us(rt1[s]) > b + 0.5))
        row.append(f"{comp:5d}/{sto:5d}")
    print(f"  {b:5.1f} " + "  ".join(row))
