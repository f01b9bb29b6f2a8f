"""Per-kernel statistics (the rocprofv3 --stats kernel table) from a rocprofv3 results database
(rocpd SQLite, the default output format of ROCm 7.2's rocprofv3):
    python tools/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys


def main(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        r = rows.setdefault(name, [0, 0, None, None])
        r[0] += 1
        r[1] += dur
        r[2] = dur if r[2] is None else min(r[2], dur)
        r[3] = dur if r[3] is None else max(r[3], dur)
    total = sum(r[1] for r in rows.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, (n, tot, lo, hi) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, n, tot, tot / n, 100.0 * tot / total, lo, hi])
            if "swarm" in name or "policy" in name:
                print(f"{name[:70]:70s} calls {n:6d} avg {tot / n / 1000:8.2f} us  {100.0 * tot / total:5.1f} %")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
