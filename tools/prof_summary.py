#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into a markdown table.

usage: tools/prof_summary.py <prefix>_kernel_stats.csv <prefix>_kernel_trace.csv [steps]
Also reports, per kernel template, the dispatches of its LARGEST grid (for the
dominant layer: k_conv_fwd<bf16,128,128> at grid 2048 x 1 = the stage-1 block-0
3x3 128->128 conv) so the bench's live HIP-event timing can be cross-checked.
"""
import csv
import sys
from collections import defaultdict


def main():
    stats, trace = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
        print(f"| `{name[:90]}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    print(f"\nTotal kernel time {tot/1e6:.1f} ms" + (f" over {steps} steps = {tot/1e6/steps:.2f} ms/step" if steps else ""))
    by = defaultdict(list)
    for r in csv.DictReader(open(trace)):
        key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("\nLongest dispatch groups (kernel, grid):")
    print("| kernel | grid | dispatches | avg us | min us | max us |")
    print("|---|---|---:|---:|---:|---:|")
    for (k, gx, gy, gz), d in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:30]:
        print(f"| `{k[:80]}` | {gx}x{gy}x{gz} | {len(d)} | {sum(d)/len(d):.1f} | {min(d):.1f} | {max(d):.1f} |")


if __name__ == "__main__":
    main()
