#!/usr/bin/env python3
"""Time acfe_mel_fwd (k_mel_w4: normalize-on-load, frame, Hann, 4096 rFFT,
|X|^2, banded mel) on the T1 batch: 512 synthetic 3 s clips at 48 kHz, 128
mels, HIP events on the launch stream, median of --iters launches; GB/s of
raw-in + mel-out bytes and fp32 VALU TFLOP/s (68.87 MFLOP per clip).
usage: python tools/mel_bench.py [--batch 512] [--iters 9]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe import frontend as fe  # noqa: E402
from acfe._lib import lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--iters", type=int, default=9)
ap.add_argument("--w5", type=int, default=None, help="acfe_mel_w5_frames(f): 0 = k_mel_w4, f = one wave per frame")
ap.add_argument("--prenorm", action="store_true",
                help="clips normalised beforehand (acfe.train.FrontEnd's path): no normalize-on-load")
a = ap.parse_args()
if a.w5 is not None:
    lib.acfe_mel_w5_frames(a.w5)
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(3)
x = (torch.rand((a.batch, 144000), generator=g) * 2 - 1).to(dev)
plan = fe.MelPlan(n_mels=128)
st = fe.normalize_stats(x)
if a.prenorm:
    x = fe.normalize_apply(x, st)
    st = None
out = plan.mel(x, st, layout="btm")
torch.cuda.synchronize()
ts = []
for _ in range(a.iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.mel(x, st, layout="btm")
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
t = sorted(ts)[len(ts) // 2]
T = out.shape[1]
byts = a.batch * (144000 * 4 + T * 128 * 4)
print(f"[w5={a.w5}] mel {a.batch} clips{' (pre-normalised)' if a.prenorm else ''}: {t:.3f} ms  {byts / t / 1e6:.1f} GB/s  {a.batch * 68.87e6 / t / 1e9:.2f} TFLOP/s "
      f"({a.batch * 68.87e6 / t / 1e9 / 157.3 * 100:.1f} % of fp32 VALU peak)", flush=True)
