#!/usr/bin/env python3
"""Static ISA census of one kernel instantiation: per-loop instruction mix (diagnostic tool).

    python tools/isa_loops.py k.s '<KIND>,<DYN>,<KS>,<MSL>,<WAVE>'
"""
import re
import sys

s = open(sys.argv[1]).read()
kind, dyn, ks, msl, wave = sys.argv[2].split(",")
name = (f"_ZN12_GLOBAL__N_112swarm_kernelILi{kind}ELi{dyn}ELi{ks}ELi{msl}ELb{wave}EEEvNS_7KParamsE"
        "11swarm_statePKfPKh9swarm_outS6_i")
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
body = s[i:j].split("\n")
labels = {}
for k, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = k


def census(seg):
    ins = [x.strip() for x in seg if x.strip() and not x.strip().startswith((";", "."))
           and not re.match(r"^\.?LBB", x.strip())]
    cnt = {}
    for x in ins:
        op = x.split()[0]
        cls = ("trans" if re.match(r"v_(sqrt|rsq|rcp|exp|log|sin|cos)_", op) else
               "f64" if re.search(r"_f64", op) else
               "valu" if op.startswith("v_") else op.split("_")[0])
        cnt[cls] = cnt.get(cls, 0) + 1
    return len(ins), cnt


tot, c = census(body)
print("whole kernel:", tot, c)
for k, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l) or re.search(r"s_branch\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < k:
        n, c = census(body[labels[m.group(1)]:k + 1])
        print(f"loop {m.group(1)} lines {labels[m.group(1)]}-{k}: {n} instr {c}")
if len(sys.argv) > 3:
    lab = sys.argv[3]
    a = labels[lab]
    for x in body[a:a + int(sys.argv[4]) if len(sys.argv) > 4 else a + 200]:
        print(x)
