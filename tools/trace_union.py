"""Step time of overlapping env-group launches from a rocprofv3 kernel trace.

    python tools/trace_union.py <run_kernel_trace.csv> [kernel-substring] [launches-per-step]

With env groups the launches of one step run concurrently on different queues, so the
per-dispatch average (--stats) is not the step time.  This takes the union of the matching
dispatches' [start, end] intervals inside each contiguous busy window and divides by the number
of steps (dispatches / launches-per-step), per window and overall; the longest window is the timed
region of bench.py (and its device warm-up).
"""
import csv
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "swarm_step64_once"
per_step = int(sys.argv[3]) if len(sys.argv) > 3 else 2
iv = []
queues = set()
with open(path) as fh:
    for r in csv.DictReader(fh):
        if pat in r["Kernel_Name"]:
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            queues.add(r["Queue_Id"])
iv.sort()
windows = []  # merged busy windows: [start, end, dispatches]
for s, e in iv:
    if windows and s <= windows[-1][1] + 2000:  # gaps under 2 us belong to the same window
        windows[-1][1] = max(windows[-1][1], e)
        windows[-1][2] += 1
    else:
        windows.append([s, e, 1])
tot_busy = sum(w[1] - w[0] for w in windows)
durs = [e - s for s, e in iv]
print(f"{len(iv)} dispatches of '{pat}' on queues {sorted(queues)}; per-dispatch mean {sum(durs) / len(durs) / 1e3:.2f} us")
print(f"busy union {tot_busy / 1e3:.1f} us over {len(windows)} windows -> {tot_busy / (len(iv) / per_step) / 1e3:.2f} us per step "
      f"({per_step} launches per step)")
big = max(windows, key=lambda w: w[2])
print(f"largest window: {big[2]} dispatches, {(big[1] - big[0]) / 1e3:.1f} us -> {(big[1] - big[0]) / (big[2] / per_step) / 1e3:.2f} us per step")
