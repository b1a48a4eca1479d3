#!/usr/bin/env python3
"""Time the acfe convolution kernels on the wr_resnet_bird T1 layer shapes
and wr_resnet's stride-1 3x3 stages (batch 512, bf16) with HIP events on the launch stream.  Prints TFLOP/s per
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
    # wr_resnet (resnet/wr_resnet.py) stage 1 / 2 / 3 stride-1 3x3 convs
    ("wrn s1 3x3 64->64", 128, 513, 64, 64, 3, 3),
    ("wrn s2 3x3 128->128", 64, 257, 128, 128, 3, 3),
    ("wrn s3 3x3 256->256", 22, 86, 256, 256, 3, 3),
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
    ap.add_argument("--layers", default="", help="comma-separated layer indices (default all)")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--no-bias", action="store_true")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad", help="subset of fwd,dgrad,wgrad")
    a = ap.parse_args()
    sel = {int(i) for i in a.layers.split(",") if i} or set(range(len(LAYERS)))
    from acfe._lib import call, lib
    from acfe._torch import ptr, stream

    dev = torch.device("cuda", 0)
    for li, (name, H, W, C, K, R, S) in enumerate(LAYERS):
        if li not in sel:
            continue
        N = a.batch
        x = (torch.randn((N, H, W, C), device=dev) * 0.5).to(torch.bfloat16)
        w = torch.randn((K, R, S, C), device=dev) / (R * S * C) ** 0.5
        b = torch.zeros(K, device=dev)
        P, pt = ops.same_padding(H, R, 1)
        Q, pl = ops.same_padding(W, S, 1)
        wp, wf = ops.pack_weights(w, torch.bfloat16, False), ops.pack_weights(w, torch.bfloat16, True)
        y = torch.empty((N, P, Q, K), dtype=torch.bfloat16, device=dev)
        dy = (torch.randn((N, P, Q, K), device=dev)).to(torch.bfloat16)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        rows = lib.acfe_conv2d_stats_rows(N * P * Q, K)
        st = torch.empty((rows, 2, wp.shape[0]), dtype=torch.float64, device=dev)
        wsz = lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, R, S, P, Q)
        ws = torch.empty((wsz,), dtype=torch.float32, device=dev)
        flops = 2.0 * N * H * W * K * R * S * C
        nan = float("nan")
        run = set(a.passes.split(","))
        t_f = nan if "fwd" not in run else timeit(lambda: call("acfe_conv2d_fwd", ptr(x), N, H, W, C, ptr(wp), K, R, S, 1, pt, pl, P, Q, None if a.no_bias else ptr(b),
                                  ptr(y), 1, None if a.no_stats else ptr(st), stream()), a.iters)
        t_d = nan if "dgrad" not in run else timeit(lambda: call("acfe_conv2d_dgrad", ptr(dy), N, P, Q, K, ptr(wf), C, R, S, 1, pt, pl, H, W,
                                  ptr(dx), 1, None, stream()), a.iters)
        t_w = nan if "wgrad" not in run else timeit(lambda: call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, R, S, 1, pt, pl, P, Q,
                                  ptr(dw), 0.0, 1, ptr(ws), stream()), a.iters)
        print(f"{name:28s} fwd {t_f:7.3f} ms {flops / t_f / 1e9:7.1f} TF | dgrad {t_d:7.3f} ms "
              f"{flops / t_d / 1e9:7.1f} TF | wgrad {t_w:7.3f} ms {flops / t_w / 1e9:7.1f} TF", flush=True)
        del x, w, y, dy, dx, dw, ws, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
