#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin):
one line per kernel with VGPRs, AGPRs, VGPR spills, scratch bytes/lane."""
import re
import sys
import subprocess

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    n = re.sub(r"\(acfe::ConvGeom.*", "", r["name"]).replace("void ", "")
    print(f"{n:60s} v{r.get('vgpr')} a{r.get('agpr')} spill{r.get('spill')} scr{r.get('scratch')}")
