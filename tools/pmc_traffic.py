#!/usr/bin/env python3
"""Fold the rocprofv3 --pmc passes of tools/pmc_traffic.sh into per-launch HBM
bytes of the dominant conv forward and write profiles/pmc_dominant_<tag>.json
(read by bench.py for roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) reports
half the bytes of wide coalesced streaming reads (16 B/lane, global_load and
LDS-DMA alike) -> doubled; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.
The raw TCC_EA0_RDREQ/WRREQ counts are kept for reference.
usage: tools/pmc_traffic.py <dir> <tag>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

KERNEL = os.environ.get("KNAME", "k_conv3x3_1w<1")


def per_dispatch(d):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    # the first dispatch is the untimed warm-up of conv_bench; keep the rest
    keys = sorted(vals)[1:] or sorted(vals)
    out = defaultdict(list)
    for k in keys:
        for c, v in vals[k].items():
            out[c].append(v)
    return {c: sum(v) / len(v) for c, v in out.items()}


def main():
    d, tag = sys.argv[1], sys.argv[2]
    pool = len(sys.argv) > 3 and sys.argv[3] == "pool"
    agg = {}
    for p in sorted(glob.glob(f"{d}/p*/")):
        agg.update(per_dispatch(p))
    fetch = agg.get("FETCH_SIZE", 0.0) * 1024 * 2       # KiB -> B, x2 gfx950 correction
    write = agg.get("WRITE_SIZE", 0.0) * 1024
    B, H, W, C, K = 512, 128, 256, 128, 128
    if pool:  # input + pooled output + 1-byte argmax per pooled output (weights negligible)
        algo = B * H * W * C * 2 + B * (H // 2) * (W // 2) * K * 3 + K * 9 * C * 2
        kern = (os.environ.get("KLABEL", "k_conv3x3_1w<1, 2, true>") +
                " (s1b0 conv21 3x3 128->128 @128x256 + 2x2 max-pool/dropout/BN-sums epilogue, batch 512)")
        src = "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes inside bench.py (tools/pmc_pool.sh)"
    else:
        algo = (B * H * W * C + B * H * W * K) * 2 + K * 9 * C * 2
        kern = "k_conv3x3_rows<128,3> (s1b0 conv21 3x3 128->128 @128x256, batch 512)"
        src = "rocprofv3 --pmc, separate passes (tools/pmc_traffic.sh), conv_bench --layers 0 --passes fwd"
    res = {
        "kernel": kern,
        "source": src,
        "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (fetch + write) / algo if algo else None,
        "raw": agg,
        "corrections": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB->B",
    }
    out = Path(__file__).resolve().parent.parent / "profiles" / f"pmc_dominant_{tag}.json"
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
