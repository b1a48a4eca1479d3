#!/usr/bin/env python3
"""In-kernel s_memtime stamps of k_conv3x3_pool1w (diagnostic build: make -C
audio-training_amd/csrc stamps): the T1 pooled conv (512 x 128 x 256,
128 -> 128, dropout 0.1, BN sums), mean per-wave cycles per tile of each step
segment.  usage: python tools/pool1w_stamps.py"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
os.environ.setdefault("ACFE_LIB", str(ROOT / "audio-training_amd" / "acfe" / "libacfe_stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acfe import ops  # noqa: E402
from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N, H, W, C, K = 512, 128, 256, 128, 128
dev = torch.device("cuda", 0)
BF = torch.bfloat16
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
w = torch.randn((K, 3, 3, C), device=dev) / (9 * C) ** 0.5
b = torch.randn((K,), device=dev) * 0.1
wp = ops.pack_weights(w, BF, False)
P, Q = H // 2, W // 2
y = torch.empty((N, P, Q, K), dtype=BF, device=dev)
am = torch.empty((N, P, Q, K), dtype=torch.uint8, device=dev)
st = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=torch.float64, device=dev)
fn = lambda: call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(am), 0.1, 77,
                  ptr(st), 1, stream())
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
fn()
e1.record()
torch.cuda.synchronize()
buf = np.zeros(4096 * 8, np.uint64)
lib.acfe_debug_pool1w_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), buf.size)
t = buf.reshape(-1, 8)[:, :6].astype(np.float64)
t = t[t.sum(1) > 0]
tiles = N * (H // 4) * (W // 64) / 256
names = ["steps (MFMA region)", "step wait", "step barrier", "restage barrier 1", "restage stores", "restage wait+barrier"]
tot = t.sum(1).mean()
print(f"{e0.elapsed_time(e1):.3f} ms, waves {len(t)}, {tiles:.0f} tiles/WG, {tot / tiles:.0f} cyc/tile")
for i, nm in enumerate(names):
    print(f"  {nm:24s} {t[:, i].mean() / tiles:8.0f} cyc/tile  ({t[:, i].mean() / tot * 100:5.1f} %)")
