#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/ (committed evidence).

    python tools/profile_summary.py r01 [gpurun_out/r01]

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --stats, names shortened),
profiles/<round>_pmc.json (per-dispatch steady-state means of the swarm kernel's counters) and
updates profiles/pmc_traffic.json, which bench.py reads for roofline.traffic: HBM bytes per launch
= 2 x FETCH_SIZE + WRITE_SIZE (KB -> B; gfx950 FETCH_SIZE tallies 128-B read requests at 64 B,
MI355X_MICROARCH.md "HBM").
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
rnd = sys.argv[1]
src = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out" / rnd
prof = ROOT / "profiles"
prof.mkdir(exist_ok=True)


def short(name: str) -> str:
    m = re.search(r"(swarm_(?:kernel|step64_once|step64)<[^>]*>)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][:120]


stats = sorted(glob.glob(str(src / "trace" / "**" / "*kernel_stats.csv"), recursive=True))
with open(stats[0]) as fh, open(prof / f"{rnd}_kernel_stats.csv", "w", newline="") as out:
    rd, wr = csv.reader(fh), csv.writer(out)
    wr.writerow(next(rd))
    for row in rd:
        wr.writerow([short(row[0])] + row[1:])
bench = json.loads((src / "bench.json").read_text().strip().splitlines()[-1])
(prof / f"{rnd}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")
kname = bench["roofline"]["kernel"]

acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(str(src / "pmc" / "p*" / "**" / "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = short(row["Kernel_Name"])
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
pmc = {}
for k, cs in acc.items():
    pmc[k] = {}
    for c, v in sorted(cs.items()):
        vv = v[len(v) // 4:] if len(v) > 8 else v  # steady state: skip reset/warmup dispatches
        pmc[k][c] = sum(vv) / len(vv)
(prof / f"{rnd}_pmc.json").write_text(json.dumps(pmc, indent=1) + "\n")
main = pmc.get(kname, {})
traffic_f = prof / "pmc_traffic.json"
traffic = json.loads(traffic_f.read_text()) if traffic_f.exists() else {}
if "FETCH_SIZE" in main and "WRITE_SIZE" in main:
    hbm = 2.0 * main["FETCH_SIZE"] * 1024 + main["WRITE_SIZE"] * 1024
    wl = f"kinematic+swarm N={bench['config']['num_drones']} E={bench['config']['envs_per_gpu']}"
    traffic[wl] = {"hbm_bytes_per_launch": hbm, "fetch_size_kb": main["FETCH_SIZE"],
                   "write_size_kb": main["WRITE_SIZE"], "kernel": kname, "round": rnd,
                   "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
                   "correction": "2 x FETCH_SIZE (gfx950 128-B reads tallied at 64 B) + WRITE_SIZE"}
    traffic_f.write_text(json.dumps(traffic, indent=1) + "\n")
    print(f"{kname}: HBM {hbm/1e6:.1f} MB/launch vs algorithmic "
          f"{bench['roofline']['algorithmic_bytes_per_launch']/1e6:.1f} MB")
for k, v in pmc.items():
    if "swarm" in k:
        print(k, {c: round(x, 1) for c, x in v.items()})
