#!/usr/bin/env python3
"""Static VALU issue-cycle census of one kernel between s_memtime stamps (diagnostic; needs a
-DSWARM_STAMPS -S listing).  Costs per wave64 instruction at 8 waves/SIMD, measured on MI355X
with tools/valu_rate4.hip: f32 add/sub/mul/fma, and/or/xor, add_u32 ~2.4 cyc; min/max/med3,
and_or/bfi, shifts, cmp/cndmask, cvt, f64, packed f32, dpp, int mul ~4.3; sqrt/rcp ~8.6.
Both sides of every branch count (an upper bound per segment).

    python tools/isa_cycles.py listing.s kernel-substring
"""
import re
import sys
from collections import Counter

FAST = ("v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_and_b32",
        "v_or_b32", "v_xor_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mov_b32", "v_not_b32")
TRANS = ("v_sqrt_f32", "v_rcp_f32", "v_rsq_f32", "v_exp_f32", "v_log_f32")
TRANS64 = ("v_sqrt_f64", "v_rcp_f64", "v_rsq_f64")


def cost(op: str) -> float:
    base = op.split("_e32")[0].split("_e64")[0].split("_dpp")[0].split("_sdwa")[0]
    if "_dpp" in op:
        return 4.3
    if base in FAST:
        return 2.4
    if base in TRANS:
        return 8.6
    if base in TRANS64:
        return 16.6
    return 4.3


s = open(sys.argv[1]).read()
pat = sys.argv[2]
lines = s.split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and pat in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
segs = [Counter()]
cyc = [0.0]
for l in lines[start + 1:end]:
    l = l.strip()
    if not l or l.startswith((";", ".")) or l.split(";")[0].strip().endswith(":"):
        continue
    op = l.split()[0]
    if op == "s_memtime":
        segs.append(Counter())
        cyc.append(0.0)
        continue
    if op.startswith("v_"):
        segs[-1][op] += 1
        cyc[-1] += cost(op)
for k, (c, y) in enumerate(zip(segs, cyc)):
    n = sum(c.values())
    top = sorted(c.items(), key=lambda kv: -kv[1] * cost(kv[0]))[:12]
    print(f"{k}: VALU {n}  cycles {y:.0f}  " + ", ".join(f"{o}x{m}({m * cost(o):.0f})" for o, m in top))
