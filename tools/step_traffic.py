#!/usr/bin/env python3
"""Fold tools/step_traffic.sh's two rocprofv3 --pmc passes into a per-kernel
HBM traffic table of one training step: FETCH_SIZE (KiB, doubled for the
gfx950 wide-read undercount, MI355X_MICROARCH.md HBM section) and WRITE_SIZE
(KiB) summed per kernel name over the profiled steps (warm-up included: the
same work) and divided by the number of steps (k_mel_w4 dispatches, one per
step); the batch generator's kernels (outside the timed step) are left out.
usage: tools/step_traffic.py <dir> <tag> [bench args]  -> profiles/r06/step_traffic_<tag>.md"""
import csv
import glob
import sys
from collections import defaultdict
from pathlib import Path

SKIP = ("roll_cuda_kernel", "rocclr_copyBuffer")


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # kernel -> dispatch -> value
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            per[name][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return per


def main():
    d, tag = sys.argv[1], sys.argv[2]
    args = sys.argv[3] if len(sys.argv) > 3 else ""
    fetch, write = load(f"{d}/p0"), load(f"{d}/p1")
    # one mel launch per step (the kernel name carries its template arguments)
    steps = max(sum(len(v) for k, v in fetch.items() if k.split("<")[0].split()[-1] == "k_mel_w4"), 1)
    rows = []
    for k in set(fetch) | set(write):
        if any(s in k for s in SKIP):
            continue
        n = max(len(fetch.get(k, {})), len(write.get(k, {})))
        rd = sum(fetch.get(k, {}).values()) * 1024 * 2 / steps / 1e9
        wr = sum(write.get(k, {}).values()) * 1024 / steps / 1e9
        rows.append((rd + wr, k, n / steps, rd, wr))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    root = Path(__file__).resolve().parent.parent
    bc = root / "BUILD_COMMIT"
    commit = bc.read_text().strip() if bc.exists() else "?"
    out = [f"# HBM traffic per kernel of one training step ({tag}; tree {commit})", "",
           f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over `bench.py --steps 2 --warmup 1 {args}`; "
           f"reads doubled (gfx950 FETCH_SIZE correction); per step = sum over the {steps} profiled steps / {steps}.",
           "", f"**Total: {tot:.1f} GB per step** (at 8 TB/s: {tot / 8:.1f} ms).", "",
           "| kernel | dispatches / step | GB read / step | GB written / step | GB per step | share |",
           "|---|---:|---:|---:|---:|---:|"]
    for t, k, n, rd, wr in rows:
        if t < 0.05:
            continue
        out.append(f"| `{k[:90]}` | {n:.0f} | {rd:.2f} | {wr:.2f} | {t:.2f} | {100 * t / tot:.1f} % |")
    p = root / "profiles" / "r06" / f"step_traffic_{tag}.md"
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text("\n".join(out) + "\n")
    print("\n".join(out[:16]))


if __name__ == "__main__":
    main()
