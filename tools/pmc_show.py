#!/usr/bin/env python3
"""Print per-dispatch counter values (last dispatch of kernels matching a
substring) from tools/pmc_groups.sh output.  usage: pmc_show.py <dir> <kernel-substr>"""
import csv, glob, sys
from collections import defaultdict
d, k = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
    v = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            v[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if v:
        last = v[sorted(v)[-1]]
        print(f.split("/")[-2], "  ".join(f"{c}={x:.4g}" for c, x in sorted(last.items())))
