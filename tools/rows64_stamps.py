#!/usr/bin/env python3
"""ACFE_CONV_DBG=8 diagnostic for wr_resnet's stage-1 K = 64 row-halo convs
(128 x 513, 64 -> 64): the BN-prologue forward with the residual Add
(acfe_conv2d_fwd_add_bn, k_conv3x3_rows<64,8,3,true,true>), the BN-prologue
forward with dropout (acfe_conv2d_fwd_bn, <64,8,4,true,true>), the plain dgrad
(<64,8,0>) and the dgrad with the BN backward sums (acfe_conv2d_dgrad_bn,
<64,8,5>): mean per-wave cycles per pipeline step of each loop segment
(s_memtime stamps of the diagnostic build, `make -C audio-training_amd/csrc
stamps`) plus the HIP-event time.
usage: python tools/rows64_stamps.py [N]"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
os.environ["ACFE_CONV_DBG"] = "8"
os.environ.setdefault("ACFE_LIB", str(ROOT / "audio-training_amd" / "acfe" / "libacfe_stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acfe import ops  # noqa: E402
from acfe._lib import call, lib  # noqa: E402
from acfe._torch import ptr, stream  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
H, W, C, K = 128, 513, 64, 64
dev = torch.device("cuda", 0)
BF = torch.bfloat16
F32 = torch.float32
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
res = (torch.randn((N, H, W, K), device=dev) * 0.5).to(BF)
w = torch.randn((K, 3, 3, C), device=dev) / (9 * C) ** 0.5
b = torch.randn((K,), device=dev) * 0.1
sc = (torch.rand(C, device=dev) + 0.5).contiguous()
sh = (torch.randn(C, device=dev) * 0.2).contiguous()
mu = (torch.randn(C, device=dev) * 0.1).contiguous()
inv = (torch.rand(C, device=dev) + 0.5).contiguous()
wp = ops.pack_weights(w, BF, False)
wr = ops.pack_weights(w, BF, True)
rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
y = torch.empty((N, H, W, K), dtype=BF, device=dev)
xo = torch.empty((N, H, W, C), dtype=BF, device=dev)
st = torch.empty((rows, 2, wp.shape[0]), dtype=torch.float64, device=dev)
dx = torch.empty((N, H, W, C), dtype=BF, device=dev)
brows = lib.acfe_conv2d_dgrad_bn_rows(N, H, W, C, K, 3, 3, 1, 1)
part = torch.empty((brows, 2, C), dtype=torch.float64, device=dev)
names = ["issue", "mfma", "epilogue", "barrier1", "restage"]
steps = -(-H // 8) * -(-W // 64) * N * (C // 64) * 3 // 256  # pipeline steps per workgroup (256 WGs)


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
          f"{tot / steps:.0f} cyc/step total (s_memtime ticks)", flush=True)
    for i, n in enumerate(names):
        print(f"  {n:10s} {t[:, i].mean() / steps:8.1f} cyc/step  {100 * t[:, i].mean() / tot:5.1f} %")


run("fwd_add_bn k_conv3x3_rows<64,8,3,true,true>",
    lambda: call("acfe_conv2d_fwd_add_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(res), 1, ptr(y),
                 ptr(st), ptr(sc), ptr(sh), 1, ptr(xo), 1, stream()))
run("fwd_bn+dropout k_conv3x3_rows<64,8,4,true,true>",
    lambda: call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st), 0.1, 5,
                 ptr(sc), ptr(sh), 1, ptr(xo), 1, stream()))
run("dgrad k_conv3x3_rows<64,8,0>",
    lambda: call("acfe_conv2d_dgrad", ptr(y), N, H, W, K, ptr(wr), C, 3, 3, 1, 1, 1, H, W, ptr(dx), 1, None,
                 stream()))
run("dgrad_bn k_conv3x3_rows<64,8,5>",
    lambda: call("acfe_conv2d_dgrad_bn", ptr(y), N, H, W, K, ptr(wr), C, 3, 3, 1, 1, 1, H, W, ptr(dx), 1, ptr(x),
                 ptr(sc), ptr(sh), ptr(mu), ptr(inv), 1, ptr(part), brows, stream()))
