#!/usr/bin/env python3
"""Time acfe_conv2d_wgrad (3x3, stride 1, bf16) on one layer shape with HIP
events on the launch stream (A/B of the halo-wgrad variants via their env
switches, e.g. ACFE_WG16_CW=64|128).
usage: python tools/wgrad_bench.py N H W C K [iters] [unpool]   (unpool: acfe_conv2d_wgrad_unpool,
the pooled gradient + argmax bytes of the 2x2 max-pool behind the conv)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N, H, W, C, K = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
unpool = len(sys.argv) > 7 and sys.argv[7] == "unpool"
dev = torch.device("cuda", 0)
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(torch.bfloat16)
dy = (torch.randn((N, H // 2 if unpool else H, W // 2 if unpool else W, K), device=dev) * 0.5).to(torch.bfloat16)
amax = torch.randint(0, 4, dy.shape, device=dev, dtype=torch.uint8)
ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=dev)
dw = torch.empty((K, 3, 3, C), device=dev)


def run():
    if unpool:
        call("acfe_conv2d_wgrad_unpool", ptr(x), N, H, W, C, ptr(dy), ptr(amax), K, 1, 1, ptr(dw), 0.0, 1, ptr(ws),
             stream())
    else:
        call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, 3, 3, 1, 1, 1, H, W, ptr(dw), 0.0, 1, ptr(ws),
             stream())


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
print(f"wgrad{' unpool' if unpool else ''} N={N} {H}x{W} C={C} K={K}: {ms * 1e3:.1f} us per call (incl. split combine), "
      f"{2 * N * H * W * 9 * C * K / ms / 1e9:.1f} TFLOP/s", flush=True)
