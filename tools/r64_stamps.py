#!/usr/bin/env python3
"""In-kernel s_memtime stamps of k_conv3x3_r64 (diagnostic build: make -C
audio-training_amd/csrc stamps) at wr_resnet's stage-1 shape (N x 128 x 513,
64 -> 64): the BN-prologue + dropout forward (PM 4), the BN-prologue +
residual forward (PM 3) and the BN-reduce dgrad (PM 5).  Prints the mean
per-wave cycles per tile of each segment and the HIP-event time per call.
usage: python tools/r64_stamps.py [N]"""
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

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
H, W, C, K = 128, 513, 64, 64
dev = torch.device("cuda", 0)
BF = torch.bfloat16
x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(BF)
res = (torch.randn((N, H, W, K), device=dev) * 0.5).to(BF)
w = torch.randn((K, 3, 3, C), device=dev) / (9 * C) ** 0.5
b = torch.randn((K,), device=dev) * 0.1
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
mu, inv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
wp = ops.pack_weights(w, BF, False)
wf = ops.pack_weights(w, BF, True)
rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
y = torch.empty((N, H, W, K), dtype=BF, device=dev)
xb = torch.empty_like(x)
st = torch.empty((rows, 2, wp.shape[0]), dtype=torch.float64, device=dev)
brows = lib.acfe_conv2d_dgrad_bn_rows(N, H, W, C, K, 3, 3, 1, 1)
part = torch.empty((brows, 2, C), dtype=torch.float64, device=dev)
fn = lib.acfe_debug_r64_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
names = ["groups rs0", "groups rs1", "groups rs2", "wait+bar rs0", "wait+bar rs1", "bar1 rs2", "restage+pack",
         "wait+bar rs2"]
tiles = N * ((H + 7) // 8) * ((W + 63) // 64)
cases = {
    "PM4 bn+dropout (conv2a)": lambda: call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y),
                                            ptr(st), 0.1, 77, ptr(sc), ptr(sh), 1, ptr(xb), 1, stream()),
    "PM3 bn+residual (conv2b)": lambda: call("acfe_conv2d_fwd_add_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b),
                                             ptr(res), 1, ptr(y), ptr(st), ptr(sc), ptr(sh), 1, ptr(xb), 1,
                                             stream()),
    "PM5 dgrad+bn reduce": lambda: call("acfe_conv2d_dgrad_bn", ptr(x), N, H, W, K, ptr(wf), C, 3, 3, 1, 1, 1, H, W,
                                        ptr(y), 1, ptr(res), ptr(sc), ptr(sh), ptr(mu), ptr(inv), 1, ptr(part),
                                        brows, stream()),
}
for name, run in cases.items():
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    fn(buf.ctypes.data, buf.size)
    a = buf.reshape(-1, 8).astype(np.float64)
    a = a[a.sum(1) > 0]
    per_wg_tiles = tiles / (a.shape[0] / 8)
    m = a.mean(0) / per_wg_tiles
    tot = m.sum()
    print(f"{name}: {e0.elapsed_time(e1):.3f} ms, {a.shape[0]} waves, {per_wg_tiles:.1f} tiles/workgroup, "
          f"{tot:.0f} stamped cycles per tile per wave")
    for n_, v in zip(names, m):
        print(f"    {n_:14s} {v:8.0f}  {100 * v / tot:5.1f} %")
