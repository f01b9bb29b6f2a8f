"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean counter value per dispatch."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if not any(s in k for s in ("swarm_kernel", "swarm_step64", "swarm_step16q", "swarm_step256", "policy_mlp")):
                    continue
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    acc = load(root)
    for k, cs in acc.items():
        print(k[:90])
        out = {}
        for c, v in sorted(cs.items()):
            # skip the first dispatches (device reset / warmup differ); use steady-state mean
            vv = v[len(v) // 4:] if len(v) > 8 else v
            out[c] = sum(vv) / len(vv)
            print(f"  {c:28s} {out[c]:.4g}  (n={len(v)})")
        print(json.dumps(out))
