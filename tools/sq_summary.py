#!/usr/bin/env python3
"""Derived SQ-counter metrics per kernel from tools/pmc_sq.sh output (last
dispatch of each matching kernel): MFMA-pipe busy share per SIMD, wave time
spent waiting, instructions per wave, LDS bank-conflict share.
usage: tools/sq_summary.py <pmc dir> <kernel substring> [...]"""
import csv
import glob
import sys
from collections import defaultdict


def last_dispatch(d, k):
    out = {}
    for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
        v = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"]:
                v[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if v:
            out.update(v[sorted(v)[-1]])
    return out


def main():
    d = sys.argv[1]
    print("| kernel | MFMA busy / SIMD | waiting / wave-time | VALU / wave | MFMA / wave | LDS instr / wave | LDS conflict / LDS active |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k in sys.argv[2:]:
        c = last_dispatch(d, k)
        if not c:
            continue
        cu = c["SQ_BUSY_CU_CYCLES"] / 256  # per CU (counter summed over the 256 CUs)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / cu if cu else 0
        wt = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        w = c.get("SQ_WAVES", 1)
        lc = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else 0
        print(f"| `{k}` | {mf:.0%} | {wt:.0%} | {c.get('SQ_INSTS_VALU', 0) / w:,.0f} | {c.get('SQ_INSTS_MFMA', 0) / w:,.0f} | "
              f"{c.get('SQ_INSTS_LDS', 0) / w:,.0f} | {lc:.0%} |")


if __name__ == "__main__":
    main()
