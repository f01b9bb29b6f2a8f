#!/usr/bin/env python3
"""Per-SIMD VALU issue time of the step kernels from PMC instruction-class counts and the
measured gfx950 per-encoding issue costs (diagnostic).

    python tools/valu_busy.py r05o [profiles/r05o_valu_rate4.txt]

Inputs: gpurun_out/<round>/pmc_<config>/ (tools/pmc_configs.sh with the SQ_INSTS_VALU_* class
counters) and the tools/valu_rate4.hip table (ns per wave-instruction per SIMD at 8 waves per
SIMD).  The PMC classes do not name encodings: SQ_INSTS_VALU_INT32 holds both the full-rate
v_and / v_or / v_xor / v_add_u32 and the half-rate v_min / v_max / v_med3 / v_and_or / shifts,
ADD/MUL/FMA_F32 hold both the scalar (full-rate) and the packed (half-rate) forms, and the
remainder (moves, compares, cndmask, DPP, f32 min/max) spans both rates.  Each class is therefore
priced at its cheapest and at its dearest member: the two columns bound the VALU issue time.
"""
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import load  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
rnd = sys.argv[1] if len(sys.argv) > 1 else "r05o"
table = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "profiles" / f"{rnd}_valu_rate4.txt"
ns = {}
for line in table.read_text().splitlines():
    m = re.match(r"^(v_\S+(?: \S+)?)\s+([\d.]+) ns per wave-instruction", line)
    if m:
        ns[m.group(1).strip()] = float(m.group(2))


def lo_hi(*names):
    v = [ns[n] for n in names]
    return min(v), max(v)


# class -> (cheapest, dearest) member, ns per wave-instruction per SIMD
PRICE = {
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
}
CONFIGS = {"headline": ("swarm_step64_once", 1024), "n16": ("swarm_step16q", 1024), "n256": ("swarm_step256", 1024)}
print(f"per-encoding issue costs: {table} ({len(ns)} encodings); v_add_f32 {ns['v_add_f32']:.3f} ns, "
      f"v_med3_u32 {ns['v_med3_u32']:.3f} ns, v_sqrt_f32 {ns['v_sqrt_f32']:.3f} ns per wave-instruction per SIMD")
for cfg, (kname, simds) in CONFIGS.items():
    acc = load(str(ROOT / "gpurun_out" / rnd / f"pmc_{cfg}"))
    ks = [k for k in acc if kname in k]
    if not ks:
        continue
    cs = acc[ks[0]]
    mean = {c: (sum(v[len(v) // 4:]) / len(v[len(v) // 4:]) if len(v) > 8 else sum(v) / len(v)) for c, v in cs.items()}
    waves = mean["SQ_WAVES"]
    total = mean["SQ_INSTS_VALU"]
    classed = sum(mean.get(c, 0.0) for c in PRICE if c != "other")
    counts = {c: mean.get(c, 0.0) for c in PRICE if c != "other"}
    counts["other"] = max(total - classed, 0.0)
    lo = sum(n * PRICE[c][0] for c, n in counts.items()) / simds * 1e-3  # us per SIMD per dispatch
    hi = sum(n * PRICE[c][1] for c, n in counts.items()) / simds * 1e-3
    print(f"\n{cfg}: {kname}, {waves:.0f} waves per dispatch ({waves / simds:.1f} per SIMD), "
          f"{total / waves:.0f} VALU per wave")
    for c, n in counts.items():
        print(f"  {c:26s} {n / waves:7.1f} per wave   {PRICE[c][0]:.3f}-{PRICE[c][1]:.3f} ns")
    print(f"  VALU issue time per SIMD per dispatch: {lo:.1f} - {hi:.1f} us "
          f"({lo / (waves / simds):.2f} - {hi / (waves / simds):.2f} us per wave)")
    print(f"  (2-cycle model at 2.4 GHz: {total / simds * 2 / 2.4e3:.1f} us)")
    dual = mean.get("SQ_ACTIVE_INST_VALU2")
    if dual is not None:
        print(f"  SQ_ACTIVE_INST_VALU2 (quad-cycles with two VALU issued, per SIMD): {dual / simds:.0f}")
