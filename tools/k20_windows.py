"""Busy windows of a short bench run from a rocprofv3 kernel trace (driver command, K = 20).

    python tools/k20_windows.py <run_kernel_trace.csv> [kernel-substring] [min-dispatches]

Prints every contiguous busy window (gaps under 2 us merged) of the matching kernel with its
dispatch count and span, and, for the last window holding at least `min-dispatches`, each
dispatch's queue, start offset and duration: how much of the timed region is pipeline fill /
drain of the env groups and how much is steady state.
"""
import csv
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "swarm_step64"
min_d = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = []
with open(path) as fh:
    for r in csv.DictReader(fh):
        if pat in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]))
rows.sort()
windows = []  # [start, end, [rows]]
for s, e, q in rows:
    if windows and s <= windows[-1][1] + 2000:
        windows[-1][1] = max(windows[-1][1], e)
        windows[-1][2].append((s, e, q))
    else:
        windows.append([s, e, [(s, e, q)]])
for i, (s, e, rs) in enumerate(windows):
    if len(rs) >= 10:
        gap = (s - windows[i - 1][1]) / 1e3 if i else 0.0
        print(f"window {i}: {len(rs)} dispatches, span {(e - s) / 1e3:.1f} us, gap before {gap:.1f} us")
cand = [w for w in windows if len(w[2]) >= min_d and len(w[2]) <= 4 * min_d]
if cand:
    s0 = cand[0][0]
    print(f"first window with {min_d}..{4 * min_d} dispatches:")
    for s, e, q in cand[0][2]:
        print(f"  q{q} start {(s - s0) / 1e3:7.1f} dur {(e - s) / 1e3:5.1f}")
