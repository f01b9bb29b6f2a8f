"""Fold rocprofv3 PMC passes of the bench configs into profiles/pmc_traffic.json (and a per-round
counter summary profiles/<round>_pmc.json).

    python tools/pmc_record.py r02        # reads gpurun_out/r02/pmc_<config>/p*/

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB units; MI355X_MICROARCH.md: gfx950
FETCH_SIZE tallies 128-B streaming reads at 64 B), the step kernel's steady-state dispatches only.
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import load  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
KEYS = {"headline": "kinematic+swarm N=64 E=8192", "n16": "kinematic+swarm N=16 E=1024",
        "n256": "kinematic+swarm N=256 E=1024 +global_state"}
ALG = {"headline": 114204672, "n16": 3658752, "n256": 63046656}


def main(rnd: str) -> None:
    traffic_f = ROOT / "profiles" / "pmc_traffic.json"
    traffic = json.loads(traffic_f.read_text()) if traffic_f.exists() else {}
    summary = {}
    for cfg, key in KEYS.items():
        acc = load(str(ROOT / "gpurun_out" / rnd / f"pmc_{cfg}"))
        step = {k: v for k, v in acc.items() if "swarm_kernel<1" not in k}  # drop the reset kernel
        if not step:
            continue
        name, cs = max(step.items(), key=lambda kv: len(kv[1].get("SQ_WAVES", [])))
        mean = {}
        for c, v in cs.items():
            vv = v[len(v) // 4:] if len(v) > 8 else v
            mean[c] = sum(vv) / len(vv)
        hbm = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
        waves = mean["SQ_WAVES"]
        short = name.replace("void ", "").replace("(anonymous namespace)::", "")
        rec = {"kernel": short.split("(")[0],
               "round": rnd, "hbm_bytes_per_launch": hbm,
               "fetch_size_kb": mean["FETCH_SIZE"], "write_size_kb": mean["WRITE_SIZE"],
               "algorithmic_bytes_per_launch": ALG[cfg],
               "valu_insts_per_launch": mean["SQ_INSTS_VALU"],
               "valu_insts_per_wave": mean["SQ_INSTS_VALU"] / waves,
               "salu_insts_per_wave": mean["SQ_INSTS_SALU"] / waves,
               "lds_insts_per_wave": mean["SQ_INSTS_LDS"] / waves,
               # bank-conflict stall cycles per LDS-instruction issue cycle: two different counters,
               # so a ratio, not a fraction (it can exceed 1)
               "lds_bank_conflict_cycles_per_lds_issue_cycle":
                   mean["SQ_LDS_BANK_CONFLICT"] / max(mean["SQ_ACTIVE_INST_LDS"], 1),
               "waves": waves,
               "correction": "2 x FETCH_SIZE (gfx950 128-B reads tallied at 64 B) + WRITE_SIZE"}
        traffic[key] = rec
        summary[cfg] = {"kernel": rec["kernel"], "counters_per_dispatch": mean}
        print(cfg, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items()}))
    traffic_f.write_text(json.dumps(traffic, indent=1) + "\n")
    (ROOT / "profiles" / f"{rnd}_pmc.json").write_text(json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
