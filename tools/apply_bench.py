#!/usr/bin/env python3
"""Time acfe_bn_bwd_apply_ex variants (dropout on / off, channel sums on / off,
residual add) on one NHWC shape, HIP events on the launch stream, with the
effective HBM rate of its streams.  usage: python tools/apply_bench.py N H W C [iters]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N, H, W, C = (int(v) for v in sys.argv[1:5])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dev = torch.device("cuda", 0)
BF = torch.bfloat16
rows = N * H * W
gy = torch.randn((rows, C), device=dev).to(BF)
x = torch.randn((rows, C), device=dev).to(BF)
add = torch.randn((rows, C), device=dev).to(BF)
dx = torch.empty((rows, C), dtype=BF, device=dev)
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
coef = torch.randn(3 * C, device=dev) * 0.5
sums = torch.empty((lib.acfe_reduce_blocks(rows), 2, C), dtype=torch.float64, device=dev)


def t(rate, with_sums, with_add):
    def f():
        call("acfe_bn_bwd_apply_ex", ptr(gy), 1, ptr(x), 1, rows, C, ptr(sc), ptr(sh), 1 | (2 if with_add else 0),
             ptr(coef), ptr(add) if with_add else None, rate, 7, ptr(dx), 1, ptr(sums) if with_sums else None,
             stream())
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    nbytes = rows * C * 2 * (4 if with_add else 3)
    print(f"apply {N}x{H}x{W}x{C} drop {rate} sums {int(with_sums)} add {int(with_add)}: {us:.1f} us, "
          f"{nbytes / us / 1e3:.0f} GB/s", flush=True)


for rate, s_, a_ in [(0.1, True, False), (0.1, False, False), (0.0, True, False), (0.0, False, False),
                     (0.0, True, True)]:
    t(rate, s_, a_)
