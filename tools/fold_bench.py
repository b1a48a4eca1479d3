#!/usr/bin/env python3
"""Time the Conv2D -> Dropout -> BN backward fold (acfe_conv2d_wgrad_bnbwd)
against its unfused chain (acfe_bn_bwd_apply_ex with dropout + channel sums,
then acfe_conv2d_wgrad), HIP events on the launch stream.
usage: python tools/fold_bench.py N H W C K [iters] [rate]   (ACFE_LIB selects a library variant)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N, H, W, C, K = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
rate = float(sys.argv[7]) if len(sys.argv) > 7 else 0.1
dev = torch.device("cuda", 0)
BF = torch.bfloat16
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
gy = (torch.randn((N, H, W, K), device=dev) * 0.5).to(BF)
u = torch.randn((N, H, W, K), device=dev).to(BF)
sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.2
coef = torch.randn(3 * K, device=dev) * 0.5
dy = torch.empty((N, H, W, K), dtype=BF, device=dev)
ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=dev)
dw = torch.empty((K, 3, 3, C), device=dev)
rows = N * H * W
sums0 = torch.empty((lib.acfe_reduce_blocks(rows), 2, K), dtype=torch.float64, device=dev)
srows = lib.acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K)
sums1 = torch.empty((max(srows, 1), 2, K), dtype=torch.float64, device=dev)


def apply():
    call("acfe_bn_bwd_apply_ex", ptr(gy), 1, ptr(u), 1, rows, K, ptr(sc), ptr(sh), 1, ptr(coef), None, rate, 7,
         ptr(dy), 1, ptr(sums0), stream())


def wgrad():
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, 3, 3, 1, 1, 1, H, W, ptr(dw), 0.0, 1, ptr(ws), stream())


def fused():
    call("acfe_conv2d_wgrad_bnbwd", ptr(x), N, H, W, C, ptr(gy), ptr(u), K, ptr(sc), ptr(sh), 1, ptr(coef), None, rate, 7,
         ptr(dy), ptr(dw), 0.0, ptr(ws), ptr(sums1), stream())


def t(f):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


ta, tw, tf = t(apply), t(wgrad), t(fused)
print(f"fold rate {rate} N={N} {H}x{W} C={C} K={K}: apply {ta:.1f} us + wgrad {tw:.1f} us = {ta + tw:.1f} us; "
      f"fused {tf:.1f} us ({tf - tw:+.1f} over the wgrad)", flush=True)
