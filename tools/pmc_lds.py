"""LDS bank-conflict attribution from tools/pmc_variants.sh runs (one line per library variant):
    python tools/pmc_lds.py <gpurun_out/tag> [kernel-substring] [variant ...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import load  # noqa: E402

root = Path(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "swarm_step64_once"
names = sys.argv[3:] or sorted(p.name[4:] for p in root.glob("pmc_*") if p.is_dir())
for v in names:
    acc = load(str(root / f"pmc_{v}"))
    for k, cs in acc.items():
        if pat not in k:
            continue
        m = {c: sum(x[len(x) // 4:]) / len(x[len(x) // 4:]) for c, x in cs.items()}
        w = m["SQ_WAVES"]
        print(f"{v:10s} VALU/wave {m['SQ_INSTS_VALU'] / w:7.0f}  LDS instr/wave {m['SQ_INSTS_LDS'] / w:6.1f}  "
              f"LDS issue cycles/wave {m['SQ_ACTIVE_INST_LDS'] / w:6.1f}  bank-conflict cycles/wave "
              f"{m['SQ_LDS_BANK_CONFLICT'] / w:5.1f}  ratio {m['SQ_LDS_BANK_CONFLICT'] / max(m['SQ_ACTIVE_INST_LDS'], 1):.3f}")
