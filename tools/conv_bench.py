#!/usr/bin/env python3
"""Time the acfe convolution kernels on the wr_resnet_bird T1 layer shapes
(batch 512, bf16) with HIP events on the launch stream.  Prints TFLOP/s per
(layer, pass).  usage: python tools/conv_bench.py [--batch 512] [--iters 5]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe import ops  # noqa: E402

# (name, H, W, C, K, R, S)
LAYERS = [
    ("s1b0.conv21 3x3 128->128", 128, 256, 128, 128, 3, 3),
    ("s1b0.conv2a0 1x1 16->128", 128, 256, 16, 128, 1, 1),
    ("s1b0.conv2b 3x3 128->64", 64, 128, 128, 64, 3, 3),
    ("s1b1.conv21 3x3 64->64", 64, 128, 64, 64, 3, 3),
    ("s2b1.conv21 3x3 128->32", 32, 64, 128, 32, 3, 3),
    ("head (4,10) 256->128", 16, 32, 256, 128, 4, 10),
]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in evs)[len(evs) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, H, W, C, K, R, S in LAYERS:
        N = a.batch
        x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(torch.bfloat16).requires_grad_(True)
        w = (torch.randn((K, R, S, C), device=dev) / (R * S * C) ** 0.5).requires_grad_(True)
        b = torch.zeros(K, device=dev, requires_grad=True)
        flops = 2.0 * N * H * W * K * R * S * C
        y, _ = ops.conv2d(x, w, b, 1, "same", want_stats=True)
        gy = torch.randn_like(y)
        t_f = timeit(lambda: ops.conv2d(x, w, b, 1, "same", want_stats=True), a.iters)
        fn_b = lambda: torch.autograd.grad(ops.conv2d(x, w, b, 1, "same")[0], (x, w), gy)  # noqa: E731
        t_fb = timeit(fn_b, a.iters)
        t_b = t_fb - timeit(lambda: ops.conv2d(x, w, b, 1, "same"), a.iters)
        print(f"{name:28s} fwd {t_f:8.3f} ms {flops / t_f / 1e9:8.1f} TF | bwd(dgrad+wgrad+db) {t_b:8.3f} ms "
              f"{2 * flops / t_b / 1e9:8.1f} TF", flush=True)
        del x, w, b, y, gy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
