#!/usr/bin/env python3
"""Per-SIMD VALU issue time of the step kernels from PMC instruction-class counts and the
measured gfx950 per-encoding issue costs (diagnostic; its numbers feed bench.py's roofline.valu).

    python tools/valu_busy.py fold <round>       # gpurun_out/<round>/pmc_<config>/ -> profiles/<round>_valu_class_pmc.jsonl
    python tools/valu_busy.py <round> [--record] # profiles/<round>_valu_class_pmc.jsonl -> table
                                                 # (--record: into profiles/pmc_traffic.json)

Inputs of the table: profiles/<round>_valu_class_pmc.jsonl (per config, the mean counters per
dispatch of the step kernel: SQ_INSTS_VALU and its SQ_INSTS_VALU_* classes, SQ_ACTIVE_INST_VALU,
SQ_WAVES) and profiles/r05o_valu_rate4.txt (tools/valu_rate4.hip: ns per wave-instruction per SIMD
at 8 waves per SIMD).  The PMC classes do not name encodings: SQ_INSTS_VALU_INT32 holds both the
full-rate v_and / v_or / v_xor / v_add_u32 and the half-rate v_min / v_max / v_med3 / v_and_or /
shifts, ADD/MUL/FMA_F32 hold both the scalar (full-rate) and the packed (half-rate) forms, and the
remainder (moves, compares, cndmask, DPP, f32 min/max) spans both rates.  Each class is therefore
priced at its cheapest and at its dearest member: the two columns bound the VALU issue time.

`--record` stores per workload: valu_class_per_wave, valu_issue_ns_per_wave [lo, hi] (per wave,
per SIMD), active_inst_valu_per_wave (SQ_ACTIVE_INST_VALU, quad-cycles) and the round, which
bench.py turns into busy fractions of its own measured step time.
"""
import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

ROOT = Path(__file__).resolve().parents[1]
RATE_TABLE = ROOT / "profiles" / "r05o_valu_rate4.txt"
CLASSES = ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
           "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
           "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_INT64")
# config -> (kernel name substring, SIMDs, pmc_traffic.json workload key)
CONFIGS = {"headline": ("swarm_step64_once", 1024, "kinematic+swarm N=64 E=8192"),
           "n16": ("swarm_step16q", 1024, "kinematic+swarm N=16 E=1024"),
           "n256": ("swarm_step256", 1024, "kinematic+swarm N=256 E=1024 +global_state")}


def prices(table: Path = RATE_TABLE) -> dict:
    ns = {}
    for line in table.read_text().splitlines():
        m = re.match(r"^(v_\S+(?: \S+)?)\s+([\d.]+) ns per wave-instruction", line)
        if m:
            ns[m.group(1).strip()] = float(m.group(2))

    def lo_hi(*names):
        v = [ns[n] for n in names]
        return min(v), max(v)

    # class -> (cheapest, dearest) member, ns per wave-instruction per SIMD
    return {
        "SQ_INSTS_VALU_INT32": lo_hi("v_add_u32", "v_xor_b32", "v_and_b32", "v_med3_u32", "v_min_u32", "v_and_or_b32",
                                     "v_lshlrev_b32", "v_mul_u32_u24"),
        "SQ_INSTS_VALU_ADD_F32": lo_hi("v_add_f32", "v_sub_f32", "v_pk_add_f32"),
        "SQ_INSTS_VALU_MUL_F32": lo_hi("v_mul_f32", "v_pk_mul_f32"),
        "SQ_INSTS_VALU_FMA_F32": lo_hi("v_fma_f32", "v_fmac_f32", "v_pk_fma_f32"),
        "SQ_INSTS_VALU_TRANS_F32": lo_hi("v_sqrt_f32", "v_rcp_f32"),
        "SQ_INSTS_VALU_CVT": lo_hi("v_cvt_f64_f32", "v_cvt_f32_f64", "v_cvt_f32_u32"),
        "SQ_INSTS_VALU_ADD_F64": lo_hi("v_add_f64"),
        "SQ_INSTS_VALU_MUL_F64": lo_hi("v_add_f64", "v_fma_f64"),
        "SQ_INSTS_VALU_FMA_F64": lo_hi("v_fma_f64"),
        "SQ_INSTS_VALU_INT64": lo_hi("v_mad_u64_u32", "v_add_f64"),
        "other": lo_hi("v_mov_b32", "v_cmp_lt_f32", "v_cndmask_e64 s", "v_add_f32_dpp", "v_min_f32", "v_max_f32"),
    }, ns


def fold(rnd: str) -> None:
    """gpurun_out/<rnd>/pmc_<config>/p*/ (rocprofv3 CSVs) -> profiles/<rnd>_valu_class_pmc.jsonl"""
    from pmc_summary import load
    out = []
    for cfg, (kname, _, _) in CONFIGS.items():
        acc = load(str(ROOT / "gpurun_out" / rnd / f"pmc_{cfg}"))
        ks = [k for k in acc if kname in k]
        if not ks:
            continue
        cs = acc[ks[0]]
        mean = {c: (sum(v[len(v) // 4:]) / len(v[len(v) // 4:]) if len(v) > 8 else sum(v) / len(v))
                for c, v in cs.items()}
        kfull = ks[0].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        out.append({"config": cfg, "kernel": kfull, **{c: round(x, 1) for c, x in sorted(mean.items())}})
    f = ROOT / "profiles" / f"{rnd}_valu_class_pmc.jsonl"
    f.write_text("".join(json.dumps(r) + "\n" for r in out))
    print(f"wrote {f} ({len(out)} configs)")


def table(rnd: str, record: bool = False) -> None:
    price, ns = prices()
    rows = [json.loads(s) for s in (ROOT / "profiles" / f"{rnd}_valu_class_pmc.jsonl").read_text().splitlines() if s]
    print(f"per-encoding issue costs: {RATE_TABLE.relative_to(ROOT)} ({len(ns)} encodings); v_add_f32 "
          f"{ns['v_add_f32']:.3f} ns, v_med3_u32 {ns['v_med3_u32']:.3f} ns, v_sqrt_f32 {ns['v_sqrt_f32']:.3f} ns "
          f"per wave-instruction per SIMD; counters: profiles/{rnd}_valu_class_pmc.jsonl")
    traffic_f = ROOT / "profiles" / "pmc_traffic.json"
    traffic = json.loads(traffic_f.read_text()) if traffic_f.exists() else {}
    for r in rows:
        cfg = r["config"]
        kname, simds, key = CONFIGS[cfg]
        waves, total = r["SQ_WAVES"], r["SQ_INSTS_VALU"]
        counts = {c: r.get(c, 0.0) for c in CLASSES}
        counts["other"] = max(total - sum(counts.values()), 0.0)
        lo = sum(n * price[c][0] for c, n in counts.items()) / waves  # ns per wave (SIMD issue time)
        hi = sum(n * price[c][1] for c, n in counts.items()) / waves
        wps = waves / simds
        print(f"\n{cfg}: {r.get('kernel', kname)}, {waves:.0f} waves per dispatch ({wps:.1f} per SIMD), "
              f"{total / waves:.0f} VALU per wave")
        for c, n in counts.items():
            print(f"  {c:26s} {n / waves:7.1f} per wave   {price[c][0]:.3f}-{price[c][1]:.3f} ns")
        print(f"  VALU issue time per SIMD per dispatch: {lo * wps * 1e-3:.1f} - {hi * wps * 1e-3:.1f} us "
              f"({lo * 1e-3:.2f} - {hi * 1e-3:.2f} us per wave)")
        print(f"  (2-cycle model at 2.4 GHz: {total / simds * 2 / 2.4e3:.1f} us)")
        act = r.get("SQ_ACTIVE_INST_VALU")
        if act is not None:
            print(f"  SQ_ACTIVE_INST_VALU: {act / waves:.0f} quad-cycles per wave = {4 * act / total:.2f} cycles per "
                  f"VALU instruction; {4 * act / simds / 1e3:.1f}k SIMD-cycles per SIMD per dispatch")
        dual = r.get("SQ_ACTIVE_INST_VALU2")
        if dual is not None:
            print(f"  SQ_ACTIVE_INST_VALU2 (quad-cycles with two VALU issued, per SIMD): {dual / simds:.0f}")
        if record and key in traffic:
            traffic[key].update({
                "valu_class_round": rnd,
                "valu_class_per_wave": {c: round(n / waves, 2) for c, n in counts.items()},
                "valu_issue_ns_per_wave": [round(lo, 2), round(hi, 2)],
                "valu_issue_price_table": str(RATE_TABLE.relative_to(ROOT)),
                **({"active_inst_valu_per_wave": round(act / waves, 2)} if act is not None else {}),
                "valu_insts_per_wave_class_pass": round(total / waves, 2),
                "simds": simds})
    if record:
        traffic_f.write_text(json.dumps(traffic, indent=1) + "\n")
        print(f"\nrecorded into {traffic_f.relative_to(ROOT)}")


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "fold":
        fold(a[1])
    else:
        table(a[0] if a else "r05y", record="--record" in a)
