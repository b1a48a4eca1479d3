#!/usr/bin/env python3
"""ACFE_CONV_DBG=8 diagnostic: run the dominant conv forward once with in-kernel
s_memtime stamps and print the mean per-wave cycles per K-tile of each loop
segment of k_conv_fwd_p."""
import ctypes, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
os.environ["ACFE_CONV_DBG"] = "8"
import numpy as np, torch
from acfe import ops
from acfe._lib import lib
li = int(sys.argv[1]) if len(sys.argv) > 1 else 0
shapes = [(512, 128, 256, 128, 128, 3, 3), (512, 16, 32, 256, 128, 4, 10)]
N, H, W, C, K, R, S = shapes[li]
dev = torch.device("cuda", 0)
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(torch.bfloat16)
w = torch.randn((K, R, S, C), device=dev) / (R * S * C) ** 0.5
for _ in range(3):
    y, st = ops.conv2d(x, w, torch.zeros(K, device=dev), 1, "same", want_stats=True)
torch.cuda.synchronize()
buf = np.zeros(4096 * 8, np.uint64)
lib.acfe_debug_conv_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), buf.size)
t = buf.reshape(-1, 8)[:, :6].astype(np.float64)
t = t[t.sum(1) > 0]
nk = (N * H * W // 256) // 256 * (R * S * C // 64)  # K-tiles per workgroup (256 WGs)
names = ["top->wait", "wait(vmcnt)", "barrier", "issue", "compute", "epilogue"]
print(f"waves {len(t)}, K-tiles/WG {nk}")
for i, n in enumerate(names):
    print(f"{n:12s} {t[:, i].mean() / nk:9.1f} cyc/K-tile  (max {t[:, i].max() / nk:9.1f})")
print(f"total        {t.sum(1).mean() / nk:9.1f}")
