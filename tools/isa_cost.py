#!/usr/bin/env python3
"""Estimated SIMD issue cost of an instruction range of a -S listing, from the measured gfx950
per-encoding throughputs (tools/valu_rate2.hip / valu_rate3.hip, >= 4 waves per SIMD, ns per
wave-instruction per SIMD).  Diagnostic only.

    python tools/isa_cost.py listing.s FIRST_LINE LAST_LINE
"""
import re
import sys
from collections import Counter

FAST = 1.05   # v_add/sub/mul_f32 (e32 or e64, modifiers ok), v_and/or/xor/add_u32, v_mov
SLOW = 1.85   # min/max/med3/min3, fma/fmac, pk_*, cmp, cndmask, cvt, f64, mul_hi/lo, shifts, bfe, readlane
TRANS = 3.45  # sqrt, rsq, rcp, exp, log
FAST_OPS = re.compile(r"^v_(add|sub|subrev|mul)_f32|^v_(and|or|xor)_b32|^v_(add|sub|subrev)_u32|^v_mov_b32|^v_not_b32")
TRANS_OPS = re.compile(r"^v_(sqrt|rsq|rcp|exp|log|sin|cos)_f32")


def cost(op):
    if not op.startswith("v_"):
        return 0.0
    if TRANS_OPS.match(op):
        return TRANS
    if FAST_OPS.match(op):
        return FAST
    return SLOW


lines = open(sys.argv[1]).read().split("\n")[int(sys.argv[2]) - 1:int(sys.argv[3])]
c = Counter()
tot = 0.0
for l in lines:
    l = l.strip()
    if not l or l.startswith((";", ".")) or l.split(";")[0].strip().endswith(":"):
        continue
    op = l.split()[0]
    c[op] += 1
    tot += cost(op)
nv = sum(n for o, n in c.items() if o.startswith("v_"))
print(f"VALU {nv}  est. issue {tot:.0f} ns-SIMD per wave  (fast-equivalents {tot / FAST:.0f})")
for o, n in c.most_common(30):
    if o.startswith("v_"):
        print(f"  {o:28s} {n:5d}  {n * cost(o):7.1f}")
