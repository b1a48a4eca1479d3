#!/usr/bin/env python3
"""ACFE_CONV_DBG=8 diagnostic for the row-halo conv kernels: run the dominant
T1 conv (acfe_conv2d_fwd_pool, 512 x 128 x 256, 128 -> 128, dropout 0.1, BN
sums; k_conv3x3_rows<128,6,1>) and its dgrad twin (acfe_conv2d_dgrad_unpool,
k_conv3x3_rows<128,6,2>) with in-kernel s_memtime stamps, and print the mean
per-wave cycles per pipeline step of each loop segment plus the HIP-event time.
usage: python tools/rows_stamps.py [N]"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
os.environ["ACFE_CONV_DBG"] = "8"
# the stamps are compiled only into the diagnostic build (make -C audio-training_amd/csrc stamps)
os.environ.setdefault("ACFE_LIB", str(ROOT / "audio-training_amd" / "acfe" / "libacfe_stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acfe import ops  # noqa: E402
from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
H, W, C, K = 128, 256, 128, 128
dev = torch.device("cuda", 0)
BF = torch.bfloat16
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
w = torch.randn((K, 3, 3, C), device=dev) / (9 * C) ** 0.5
b = torch.randn((K,), device=dev) * 0.1
wp = ops.pack_weights(w, BF, False)
wr = ops.pack_weights(w, BF, True)
P, Q = H // 2, W // 2
rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
y = torch.empty((N, P, Q, K), dtype=BF, device=dev)
am = torch.empty((N, P, Q, K), dtype=torch.uint8, device=dev)
st = torch.empty((rows, 2, wp.shape[0]), dtype=torch.float64, device=dev)
dx = torch.empty((N, H, W, C), dtype=BF, device=dev)
names = ["issue", "mfma", "epilogue", "barrier1", "restage"]
TR = 6 if os.environ.get("ACFE_ROWS_XRES") == "0" else 4  # K = 128 tile rows (chunk-resident 4-row default)
steps = -(-H // TR) * (W // 64) * N * (C // 64) * 3 // 256  # pipeline steps per workgroup (256 WGs)


def run(tag, fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    lib.acfe_debug_conv_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), buf.size)
    t = buf.reshape(-1, 8)[:, :5].astype(np.float64)
    t = t[t.sum(1) > 0]
    tot = t.sum(1).mean()
    print(f"{tag}: {e0.elapsed_time(e1):.3f} ms, waves {len(t)}, ~{steps} steps/WG, "
          f"{tot / steps:.0f} cyc/step total (s_memtime ticks)")
    for i, n in enumerate(names):
        print(f"  {n:10s} {t[:, i].mean() / steps:8.1f} cyc/step  {100 * t[:, i].mean() / tot:5.1f} %")


run(f"fwd_pool k_conv3x3_rows<128,{TR},1>",
    lambda: call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(am), 0.1, 7,
                 ptr(st), 1, stream()))
run(f"dgrad_unpool k_conv3x3_rows<128,{TR},2>",
    lambda: call("acfe_conv2d_dgrad_unpool", ptr(y), ptr(am), N, H, W, K, ptr(wr), C, 1, 1, ptr(dx), 1, stream()))
