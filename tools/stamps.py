"""Per-phase cycle profile of the step kernel from s_memtime stamps (diagnostic build).

Build:  hipcc ... -DSWARM_STAMPS -> build/stamps/libswarm_stamps.so   (tools/stamps.py build)
Run:    SWARM_MI355X_LIB=build/stamps/libswarm_stamps.so python tools/stamps.py run [E] [N]
"""
import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LIB = Path(os.environ.get("SWARM_STAMPS_LIB", ROOT / "build" / "stamps" / "libswarm_stamps.so"))
NAMES = ["load", "integrate", "pairs+obst", "topk", "reward", "reset", "writeback", "obs"]
if os.environ.get("SWARM_STAMPS_KERNEL") == "n256":  # swarm_step256's STAMP256 phases (wave 0)
    NAMES = ["load", "integ+put", "pass1+obst", "handover", "reward", "reset", "keys+finish", "wb+obs"]

if sys.argv[1] == "build":
    LIB.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    "-fno-slp-vectorize", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
                    "-I", str(ROOT / "include"), "-DSWARM_STAMPS", "-DSWARM_DEV_HOT", *sys.argv[2:],
                    str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_kernel.hip"),
                    str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_policy.hip"),
                    str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_eval.hip"),
                    "-o", str(LIB)], check=True)
    sys.exit(0)

os.environ["SWARM_MI355X_LIB"] = str(LIB)
sys.path.insert(0, str(ROOT / "multi-agent-rl-for-autonomous-drone-swarms_amd"))
import numpy as np
import torch
from swarm_marl_amd import VecSwarm
from swarm_marl_amd import _native as nat

e = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
n = int(sys.argv[3]) if len(sys.argv) > 3 else 64
dyn = os.environ.get("SWARM_STAMPS_DYNAMICS", "kinematic")
vec = VecSwarm(e, {"num_drones": n}, device="cuda:0", auto_reset=True, seed=0, dynamics=dyn)
vec.reset()
lib = nat.load_library()
lib.swarm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
g = torch.Generator(device="cuda:0").manual_seed(1)
acts = [torch.rand((e, n, 3), device="cuda:0", generator=g) * 2 - 1 for _ in range(4)]
for k in range(20):
    vec.step(acts[k % 4])
torch.cuda.synchronize()
blocks = e  # one stamp record per env
buf = np.zeros(min(blocks, 1 << 16) * 16, np.uint64)
lib.swarm_debug_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(-1, 16)[:, :9].astype(np.int64)
dump = os.environ.get("SWARM_STAMPS_DUMP")
if dump:
    np.savez_compressed(dump, stamps=buf.reshape(-1, 16), env_done=vec.env_done.cpu().numpy(),
                        active=vec.active.cpu().numpy())
d = np.diff(st, axis=1)
t0 = st[:, 0].min()
print(f"E={e} N={n} blocks={blocks}: wave lifetime cycles mean {np.mean(st[:,8]-st[:,0]):.0f} "
      f"median {np.median(st[:,8]-st[:,0]):.0f}; kernel span {st[:,8].max()-t0} cycles; "
      f"start spread {st[:,0].max()-t0}")
for i, nm in enumerate(NAMES):
    print(f"  {nm:12s} mean {d[:, i].mean():9.0f}  median {np.median(d[:, i]):9.0f}  p90 {np.percentile(d[:, i], 90):9.0f}")

# ---- residency census: concurrent waves per CU from (start, end) stamps and HW_ID / XCC_ID
hw = buf.reshape(-1, 16)[:, 9].astype(np.int64)
xcc = buf.reshape(-1, 16)[:, 10].astype(np.int64) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 0x1
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
best = []
for k in np.unique(key):
    idx = np.nonzero(key == k)[0]
    ev = sorted([(st[i, 0], 1) for i in idx] + [(st[i, 8], -1) for i in idx])
    c = m = 0
    for _, dlt in ev:
        c += dlt
        m = max(m, c)
    best.append((m, len(idx)))
best = np.array(best)
print(f"CUs seen {len(best)}; waves per CU total mean {best[:,1].mean():.1f}; "
      f"max concurrent waves per CU: mean {best[:,0].mean():.1f} max {best[:,0].max()} min {best[:,0].min()}")
print("simd histogram", np.bincount(simd, minlength=4))

rt0 = buf.reshape(-1, 16)[:, 11].astype(np.int64)
rt1 = buf.reshape(-1, 16)[:, 12].astype(np.int64)
clk = (st[:, 8] - st[:, 0]) / np.maximum(rt1 - rt0, 1) * 100e6
print(f"in-kernel clock (memtime/memrealtime): median {np.median(clk)/1e9:.2f} GHz")
print(f"kernel span from realtime: {(rt1.max() - rt0.min())/100:.1f} us; wave life median {np.median(rt1-rt0)/100:.2f} us, "
      f"p90 {np.percentile(rt1-rt0, 90)/100:.2f} us")
spans = []
for k in np.unique(key):
    idx = np.nonzero(key == k)[0]
    spans.append((rt1[idx].max() - rt0[idx].min()) / 100)
print(f"per-CU span us: mean {np.mean(spans):.1f} max {np.max(spans):.1f}; first start spread {(rt0.max()-rt0.min())/100:.1f} us")
order = np.argsort(rt0)
print("start times (us) of block quantiles:", [(round((rt0[order[int(q*(len(order)-1))]]-rt0.min())/100, 1)) for q in (0, .25, .5, .75, 1)])

life = (rt1 - rt0) / 100
o = np.argsort(-life)[:12]
print("longest waves: block, start_us, life_us, phase cycles [load integ pairs topk reward reset wb obs]")
for i in o:
    print(f"  {i:5d} {(rt0[i]-rt0.min())/100:7.1f} {life[i]:7.1f} {d[i].tolist()}")
print("life quantiles us:", np.percentile(life, [50, 90, 99, 99.9, 100]).round(1).tolist())

# ---- timeline: waves alive and waves in each phase, per 2-us bin (realtime clock, 100 MHz)
mt = buf.reshape(-1, 16)[:, :9].astype(np.int64)
toff = rt0 - (mt[:, 0] * 100e6 / (clk + 1e-9)).astype(np.int64)  # per-wave realtime offset of memtime 0
ph_rt = ((mt - mt[:, :1]) / (clk[:, None] / 100e6) + rt0[:, None] - rt0.min()) / 100.0  # us
bins = np.arange(0, np.ceil(ph_rt.max()) + 2, 2.0)
print("timeline (us bin: alive | load integ pairs topk reward reset wb obs)")
for b0 in bins[:-1]:
    mid = b0 + 1.0
    alive = int(((ph_rt[:, 0] <= mid) & (ph_rt[:, 8] > mid)).sum())
    inph = [int(((ph_rt[:, i] <= mid) & (ph_rt[:, i + 1] > mid)).sum()) for i in range(8)]
    print(f"  {b0:5.0f}: {alive:5d} | " + " ".join(f"{x:5d}" for x in inph))
