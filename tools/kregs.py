#!/usr/bin/env python3
"""Register/scratch census per kernel instantiation from a `hipcc -S` listing (diagnostic)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    f = dict(re.findall(r"\.amdhsa_(next_free_vgpr|next_free_sgpr|private_segment_fixed_size|accum_offset) (\d+)", body))
    t = re.search(r"swarm_kernelILi(\d)ELi(\d)ELi(\d+)ELi(\d+)ELb(\d)", name)
    print(t.groups() if t else name, f)
