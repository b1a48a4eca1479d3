#!/usr/bin/env python3
"""Fold the passes of tools/pmc_evidence.sh into
profiles/pmc_dominant_<key>_<round>.json (HBM bytes per launch: FETCH_SIZE x2
for the gfx950 wide-read undercount + WRITE_SIZE, KiB -> B, MI355X_MICROARCH.md
HBM section; averaged over the kernel's dispatches after the first) and
profiles/sq_dominant_<key>_<round>.json (SQ counters of the last dispatch:
MFMA-pipe busy per SIMD, share of wave time waiting, VALU per MFMA, LDS
bank-conflict share; formulas of tools/sq_summary.py).
usage: tools/pmc_fold.py <dir> <kernel regex> <key> <round> <algorithmic bytes> <label> <bench args>
                         [period:index]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


SELECT = None  # (period, index): keep dispatch i of every `period` consecutive ones


def dispatches(d, rx):
    """Counters per dispatch of the kernels matching rx.  The same kernel also
    runs other layers of the model: with SELECT only the dominant layer's
    dispatches are kept (its position among each step's dispatches of the
    kernel, in dispatch order; the grid size does not tell layers apart for the
    grid-stride kernels)."""
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if re.search(rx, r["Kernel_Name"]):
                vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if SELECT:
        per, idx = SELECT
        keep = sorted(vals)[idx::per]
        vals = {k: vals[k] for k in keep}
    return vals


def main():
    global SELECT
    d, rx, key, rnd, algo, label, args = sys.argv[1:8]
    if len(sys.argv) > 8 and sys.argv[8]:
        SELECT = tuple(int(v) for v in sys.argv[8].split(":"))
    algo = float(algo)
    root = Path(__file__).resolve().parent.parent
    prof = root / "profiles"
    # the tree the counters were measured on (tools/gpurun.sh writes it before
    # the snapshot travels: the GPU box has no .git)
    bc = root / "BUILD_COMMIT"
    commit = bc.read_text().strip() if bc.exists() else None
    traffic = {}
    for i, c in ((0, "FETCH_SIZE"), (1, "WRITE_SIZE")):
        v = dispatches(f"{d}/p{i}", rx)
        ks = sorted(v)[1:] or sorted(v)
        traffic[c] = sum(v[k][c] for k in ks) / max(len(ks), 1)
        traffic[c + "_dispatches"] = len(ks)
    fetch, write = traffic["FETCH_SIZE"] * 1024 * 2, traffic["WRITE_SIZE"] * 1024
    pmc = {"kernel": label, "kernel_regex": rx, "bench_args": args, "dispatch_select": SELECT,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes inside the bench command "
                     "(tools/pmc_evidence.sh)",
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
           "algorithmic_bytes_per_launch": algo, "traffic_over_algorithmic": (fetch + write) / algo,
           "raw": traffic, "corrections": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB->B",
           "commit": commit}
    (prof / f"pmc_dominant_{key}_{rnd}.json").write_text(json.dumps(pmc, indent=1) + "\n")
    c = {}
    for i in (2, 3):
        v = dispatches(f"{d}/p{i}", rx)
        if v:
            c.update(v[sorted(v)[-1]])
    cu = c["SQ_BUSY_CU_CYCLES"] / 256
    sq = {"kernel": label, "kernel_regex": rx, "bench_args": args, "dispatch_select": SELECT,
          "source": f"rocprofv3 --pmc, two passes inside the bench command (tools/pmc_evidence.sh); raw: {d}",
          "mfma_busy_per_simd": round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / cu, 4),
          "wave_time_waiting": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
          "valu_insts_per_mfma": round(c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_INSTS_MFMA", 1), 1), 3),
          "valu_insts_per_wave": round(c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1), 1),
          "lds_bank_conflict_share": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1), 3),
          "raw": c, "commit": commit}
    (prof / f"sq_dominant_{key}_{rnd}.json").write_text(json.dumps(sq, indent=1) + "\n")
    print(json.dumps({"traffic": pmc["hbm_bytes_per_launch"], "over_algo": round(pmc["traffic_over_algorithmic"], 3),
                      **{k: sq[k] for k in ("mfma_busy_per_simd", "wave_time_waiting", "valu_insts_per_mfma",
                                            "lds_bank_conflict_share")}}))


if __name__ == "__main__":
    main()
