"""Timeline of the short timed regions (the driver's K = 20) from a rocprofv3 kernel trace.

    python tools/region_trace.py <run_kernel_trace.csv> [kernel-substring] [dispatches-per-region]

Splits the step dispatches into busy windows (gaps > 20 us between windows), keeps those with
exactly `dispatches-per-region` dispatches (K steps x groups: 40 for the driver's command), and
prints per window: its span, span / K, the first step's and the last step's durations, and how
the env groups' launches sit against each other (the phase of group 1's starts inside group 0's
launches: 0 = in lock-step, 0.5 = half a launch apart).
"""
import csv
import statistics
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "swarm_step64_once"
per_region = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = []
with open(path) as fh:
    for r in csv.DictReader(fh):
        if pat in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]))
rows.sort()
wins, cur = [], []
for s, e, q in rows:
    if cur and s > max(x[1] for x in cur) + 20000:
        wins.append(cur)
        cur = []
    cur.append((s, e, q))
if cur:
    wins.append(cur)
print(f"{len(rows)} dispatches, {len(wins)} windows; sizes {[len(w) for w in wins][:12]}")
for wi, w in enumerate(wins):
    if len(w) != per_region:
        continue
    t0 = w[0][0]
    t1 = max(x[1] for x in w)
    queues = sorted({q for _, _, q in w})
    byq = {q: [(s - t0, e - t0) for s, e, qq in w if qq == q] for q in queues}
    k = len(w) // len(queues)
    durs = [e - s for s, e, _ in w]
    line = (f"window {wi}: span {(t1 - t0) / 1e3:.1f} us = {(t1 - t0) / k / 1e3:.2f} us/step over {k} steps; "
            f"dispatch mean {statistics.mean(durs) / 1e3:.1f} us")
    if len(queues) == 2:
        a, b = byq[queues[0]], byq[queues[1]]
        if a[0][0] > b[0][0]:
            a, b = b, a
        phases = []
        for s, _ in b:
            for s0, e0 in a:
                if s0 <= s < e0:
                    phases.append((s - s0) / (e0 - s0))
                    break
        line += (f"; first launches {(a[0][1] - a[0][0]) / 1e3:.1f} / {(b[0][1] - b[0][0]) / 1e3:.1f} us, "
                 f"last {(a[-1][1] - a[-1][0]) / 1e3:.1f} / {(b[-1][1] - b[-1][0]) / 1e3:.1f} us; "
                 f"group-1 start phase in group-0 launches: "
                 + " ".join(f"{p:.2f}" for p in phases[:20]))
    print(line)
