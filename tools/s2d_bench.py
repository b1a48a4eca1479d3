#!/usr/bin/env python3
"""Time wr_resnet's strided dgrads (acfe_conv2d_dgrad at stride 2 / 3, the
super-pixel path or, with ACFE_DGRAD_S2D=0, the phase path) beside the plain
stride-1 forward of the same GEMM (dY with the Mr x Ms window -> st^2 C or C
output channels, NHWC store), HIP events on the launch stream, batch 512.
usage: python tools/s2d_bench.py [iters]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe import ops  # noqa: E402
from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
BF = torch.bfloat16
N = 512


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


for name, H, W, C, K, R, st in [("s2 3x3", 128, 513, 64, 128, 3, 2), ("s3 3x3", 64, 257, 128, 256, 3, 3),
                                ("s2 1x1", 128, 513, 64, 128, 1, 2), ("s3 1x1", 64, 257, 128, 256, 1, 3)]:
    if R == 3:
        P, pt = ops.same_padding(H, 3, st)
        Q, pl = ops.same_padding(W, 3, st)
    else:
        P, Q, pt, pl = ops.valid_out(H, 1, st), ops.valid_out(W, 1, st), 0, 0
    w = torch.randn((K, R, R, C), device=dev) * 0.05
    dy = (torch.randn((N, P, Q, K), device=dev) * 0.5).to(BF)
    wf = ops.pack_weights(w, BF, True)
    dx = torch.empty((N, H, W, C), dtype=BF, device=dev)
    nb = lib.acfe_conv2d_dgrad_workspace(N, P, Q, K, C, R, R, st, pt, pl, H, W, 1)
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    td = t(lambda: call("acfe_conv2d_dgrad", ptr(dy), N, P, Q, K, ptr(wf), C, R, R, st, pt, pl, H, W, ptr(dx), 1,
                        ptr(ws), stream()))
    # the same GEMM as a plain stride-1 forward (window mr x ms, NHWC output)
    mr = -(-R // st)
    kout = C if R == 1 else st * st * C
    U, V = -(-(H + pt) // st), -(-(W + pl) // st)
    wg = torch.randn((kout, mr, mr, K), device=dev) * 0.05
    wp = ops.pack_weights(wg, BF, False)
    y = torch.empty((N, U, V, kout), dtype=BF, device=dev)
    tf = t(lambda: call("acfe_conv2d_fwd", ptr(dy), N, P, Q, K, ptr(wp), kout, mr, mr, 1, mr - 1, mr - 1, U, V,
                        None, ptr(y), 1, None, stream()))
    fl = 2.0 * N * U * V * kout * mr * mr * K
    gb = (dx.numel() + dy.numel()) * 2 / 1e9
    print(f"{name}: dgrad {td:8.1f} us ({gb / td * 1e3:6.2f} TB/s of dX + dY)   plain fwd of the same GEMM "
          f"{tf:8.1f} us ({fl / tf / 1e6:7.1f} TFLOP/s, {y.numel() * 2 / 1e9:.2f} GB out)")
