#!/usr/bin/env python3
"""Write profiles/sq_dominant_<tag>.json (read by bench.py for roofline.counters)
from a tools/pmc_sq.sh output directory: the SQ counters of the last dispatch of
the dominant kernel and the derived MFMA-busy / waiting / VALU-per-MFMA / LDS
conflict shares (formulas as tools/sq_summary.py).
usage: tools/sq_json.py <pmc dir> <kernel substring> <tag>"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from sq_summary import last_dispatch  # noqa: E402

d, k, tag = sys.argv[1], sys.argv[2], sys.argv[3]
c = last_dispatch(d, k)
cu = c["SQ_BUSY_CU_CYCLES"] / 256
res = {
    "kernel": k + " (dominant T1 forward)",
    "source": f"rocprofv3 --pmc, two passes inside bench.py (tools/pmc_sq.sh); raw: {d}",
    "mfma_busy_per_simd": round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / cu, 4),
    "wave_time_waiting": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
    "valu_insts_per_mfma": round(c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_INSTS_MFMA", 1), 1), 3),
    "lds_bank_conflict_share": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1), 3),
    "gpu_busy_cycles_per_xcd": c.get("GRBM_GUI_ACTIVE", 0) / 8,
    "raw": c,
}
out = Path(__file__).resolve().parent.parent / "profiles" / f"sq_dominant_{tag}.json"
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps({x: res[x] for x in ("mfma_busy_per_simd", "wave_time_waiting", "valu_insts_per_mfma",
                                       "lds_bank_conflict_share")}))
