#!/usr/bin/env python3
"""Static instruction census of one kernel between s_memtime stamps (diagnostic; needs a
-DSWARM_STAMPS -S listing).  Both sides of a branch count, so read it as an upper bound.

    python tools/isa_phases.py listing.s [kernel-substring]
"""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "ILi0ELi0ELi4ELi5ELi2E"
lines = s.split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and pat in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
segs = [Counter()]
for l in lines[start + 1:end]:
    l = l.strip()
    if not l or l.startswith((";", ".")) or l.split(";")[0].strip().endswith(":"):
        continue
    op = l.split()[0]
    if op == "s_memtime":
        segs.append(Counter())
        continue
    cls = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") else "LDS" if op.startswith("ds_")
           else "VMEM" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    segs[-1][cls] += 1
    segs[-1][op] += 1
for k, c in enumerate(segs):
    top = [(o, n) for o, n in c.most_common() if o not in ("VALU", "SALU", "LDS", "VMEM")][:14]
    print(k, {x: c[x] for x in ("VALU", "SALU", "LDS", "VMEM")}, top)
