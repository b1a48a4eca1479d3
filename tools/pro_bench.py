#!/usr/bin/env python3
"""Cost of the normalised-input store of the BN-prologue forwards: time
acfe_conv2d_fwd_bn (dropout + BN sums) and acfe_conv2d_fwd_add_bn (residual
Add + ReLU + BN sums) at a 64 -> 64 3x3 layer with and without x_bn_out (the
x' = ReLU(BN(x)) tile the weight gradient reads), HIP events on the launch
stream.  usage: python tools/pro_bench.py [N H W] [iters]   (default wr_resnet
stage 1: 512 128 513)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe import ops  # noqa: E402
from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N, H, W = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (512, 128, 513)
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
C = K = 64
dev = torch.device("cuda", 0)
BF = torch.bfloat16
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
r = (torch.randn((N, H, W, K), device=dev) * 0.5).to(BF)
w = torch.randn((K, 3, 3, C), device=dev) * 0.05
b = torch.randn((K,), device=dev) * 0.1
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
wp = ops.pack_weights(w, BF, False)
y = torch.empty((N, H, W, K), dtype=BF, device=dev)
xo = torch.empty((N, H, W, C), dtype=BF, device=dev)
st = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=torch.float64, device=dev)


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


for name, out in (("with x' store", xo), ("without", None)):
    td = t(lambda: call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st), 0.1, 7,
                        ptr(sc), ptr(sh), 1, ptr(out) if out is not None else None, 1, stream()))
    ta = t(lambda: call("acfe_conv2d_fwd_add_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(r), 1, ptr(y),
                        ptr(st), ptr(sc), ptr(sh), 1, ptr(out) if out is not None else None, 1, stream()))
    print(f"N={N} {H}x{W} 64->64 {name}: fwd_bn (dropout + sums) {td:8.1f} us, fwd_add_bn (add + ReLU + sums) {ta:8.1f} us")
