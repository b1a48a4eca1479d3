#!/usr/bin/env python3
"""ACFE_CONV_DBG=8 diagnostic for the persistent GEMM k_conv_fwd_p on the
wr_resnet layers it serves at batch N (default 512): per-wave s_memtime cycle
totals of its loop segments (loop top, vmcnt wait, barrier, stage issue,
LDS fragment reads + MFMA, epilogue), with the HIP-event time of the launch.
usage: python tools/fwdp_stamps.py [N]"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
os.environ["ACFE_CONV_DBG"] = "8"
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acfe import ops  # noqa: E402
from acfe._lib import lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
BF = torch.bfloat16
NAMES = ["top", "wait", "barrier", "issue", "mfma", "epilogue"]


def run(tag, fn, flops):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    buf = np.zeros(4096 * 8, np.uint64)
    lib.acfe_debug_conv_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), buf.size)
    t = buf.reshape(-1, 8)[:, :6].astype(np.float64)
    t = t[t.sum(1) > 0]
    tot = t.sum(1).mean()
    print(f"{tag}: {ms:.3f} ms ({flops / ms / 1e9:.0f} TFLOP/s), {len(t)} waves, {tot:.0f} cycles per wave")
    for i, n in enumerate(NAMES):
        print(f"    {n:9s} {100 * t[:, i].mean() / tot:5.1f} %")


def conv(H, W, C, K, R, S, st, stats, drop=None):
    x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
    w = torch.randn((K, R, S, C), device=dev) / (R * S * C) ** 0.5
    b = torch.zeros((K,), device=dev)
    P, pt = ops.same_padding(H, R, st)
    Q, pl = ops.same_padding(W, S, st)
    fl = 2.0 * N * P * Q * K * R * S * C
    lbl = f"{R}x{S}/{st} {C}->{K} @{H}x{W}"
    run(f"fwd   {lbl}" + (" + dropout" if drop else ""), lambda: ops._conv_fwd(x, w, b, st, pt, pl, P, Q, stats, drop), fl)
    dy = (torch.randn((N, P, Q, K), device=dev) * 0.5).to(BF)
    run(f"dgrad {lbl}", lambda: ops._conv_bwd(x, w, dy, st, pt, pl, P, Q, True, False, False), fl)


conv(128, 513, 64, 128, 3, 3, 2, True, (0.1, 7))    # stage-2 transition conv (b3.conv2a)
conv(128, 513, 64, 128, 1, 1, 2, False)   # its 1x1 shortcut
conv(64, 257, 128, 256, 3, 3, 3, True, (0.1, 7))    # stage-3 transition conv (stride 3)
conv(64, 257, 128, 256, 1, 1, 3, False)
conv(22, 86, 256, 256, 3, 3, 1, True)     # stage-3 3x3 (reference point: 36 K-tiles)
