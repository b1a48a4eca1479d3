#!/usr/bin/env python3
"""Time the fused T1 conv nodes at batch 512 (HIP events on the launch stream):
acfe_conv2d_fwd_pool (dropout 0.1 + BN sums), acfe_conv2d_dgrad_unpool,
acfe_conv2d_wgrad_unpool on the stage-1 block-0 3x3 128->128 @ 128x256 layer,
and acfe_conv2d_fwd_add / acfe_conv2d_fwd_dropout on the 64x128 layers.
Also checks that two launches give identical outputs (determinism).
usage: python tools/rows_bench.py [--batch 512] [--iters 7]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

from acfe import ops  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=7)
    ap.add_argument("--only", default="", help="comma list of pool,unpool,wunpool,add,drop64,wg64,wu64,wg32")
    a = ap.parse_args()
    from acfe._lib import call, lib
    from acfe._torch import ptr, stream

    only = set(x for x in a.only.split(",") if x)
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    N = a.batch
    res = {}

    def report(name, flops, fn, outs):
        t = timeit(fn, a.iters)
        first = [o.clone() for o in outs]
        fn()
        torch.cuda.synchronize()
        det = all(torch.equal(f, o) for f, o in zip(first, outs))
        res[name] = t
        print(f"{name:40s} {t:8.3f} ms {flops / t / 1e9:8.1f} TF  deterministic={det}", flush=True)

    # stage-1 block-0 conv21: 128 -> 128 @ 128 x 256, 2x2 pool
    H, W, C, K = 128, 256, 128, 128
    g = torch.Generator(device="cpu").manual_seed(1)
    flops = 2.0 * N * H * W * K * 9 * C
    if not only or only & {"pool", "unpool", "wunpool"}:
        x = (torch.randn((N, H, W, C), generator=g) * 0.5).to(bf).to(dev)
        w = (torch.randn((K, 3, 3, C), generator=g) / (9 * C) ** 0.5).to(dev)
        b = torch.zeros(K, device=dev)
        wp, wf = ops.pack_weights(w, bf, False), ops.pack_weights(w, bf, True)
        P, Q = H // 2, W // 2
        y = torch.empty((N, P, Q, K), dtype=bf, device=dev)
        am = torch.empty((N, P, Q, K), dtype=torch.uint8, device=dev)
        st = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=torch.float64, device=dev)
        if not only or "pool" in only:
            report("fwd_pool 3x3 128->128 @128x256", flops,
                   lambda: call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(am),
                                0.1, 77, ptr(st), 1, stream()), [y, am])
        gp = torch.randn((N, P, Q, K), generator=g).to(bf).to(dev)
        amr = torch.randint(0, 4, (N, P, Q, K), generator=g, dtype=torch.uint8).to(dev)
        dx = torch.empty_like(x)
        if not only or "unpool" in only:
            report("dgrad_unpool 3x3 128->128 @128x256", flops,
                   lambda: call("acfe_conv2d_dgrad_unpool", ptr(gp), ptr(amr), N, H, W, K, ptr(wf), C, 1, 1, ptr(dx), 1,
                                stream()), [dx])
        if not only or "wunpool" in only:
            ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=dev)
            dw = torch.empty((K, 3, 3, C), device=dev)
            report("wgrad_unpool 3x3 128->128 @128x256", flops,
                   lambda: call("acfe_conv2d_wgrad_unpool", ptr(x), N, H, W, C, ptr(gp), ptr(amr), K, 1, 1, ptr(dw),
                                0.0, 1, ptr(ws), stream()), [dw])
            del ws, dw
        del x, y, am, st, gp, amr, dx
        torch.cuda.empty_cache()
    # 64 x 128 layers: conv2b 128->64 + add, and 64->64 conv21 (+dropout, BN sums)
    H, W = 64, 128
    for C, K, kind in ((128, 64, "add"), (64, 64, "add"), (64, 64, "drop64"), (64, 64, "wg64"), (128, 64, "wu64"), (128, 32, "wg32")):
        if only and kind not in only:
            continue
        flops = 2.0 * N * H * W * K * 9 * C
        x = (torch.randn((N, H, W, C), generator=g) * 0.5).to(bf).to(dev)
        w = (torch.randn((K, 3, 3, C), generator=g) / (9 * C) ** 0.5).to(dev)
        b = torch.zeros(K, device=dev)
        wp = ops.pack_weights(w, bf, False)
        y = torch.empty((N, H, W, K), dtype=bf, device=dev)
        st = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=torch.float64, device=dev)
        if kind == "add":
            sc = torch.randn((N, H, W, K), generator=g).to(bf).to(dev)
            report(f"fwd_add 3x3 {C}->{K} @64x128", flops,
                   lambda: call("acfe_conv2d_fwd_add", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(sc), 1, ptr(y),
                                ptr(st), 1, stream()), [y])
            del sc
        elif kind == "wu64":  # s2 b0 branch21 128 -> 64 weight gradient from the pooled gradient
            ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=dev)
            dw = torch.empty((K, 3, 3, C), device=dev)
            gp = torch.randn((N, H // 2, W // 2, K), generator=g).to(bf).to(dev)
            amr = torch.randint(0, 4, (N, H // 2, W // 2, K), generator=g, dtype=torch.uint8).to(dev)
            report(f"wgrad_unpool 3x3 {C}->{K} @64x128", flops,
                   lambda: call("acfe_conv2d_wgrad_unpool", ptr(x), N, H, W, C, ptr(gp), ptr(amr), K, 1, 1, ptr(dw),
                                0.0, 1, ptr(ws), stream()), [dw])
            del ws, dw, gp, amr
        elif kind == "wg64" or kind == "wg32":  # 64 -> 64 @ 64x128, 128 -> 32 @ 32x64 (stage-2 branch21)
            if kind == "wg32":
                H, W = 32, 64
                flops = 2.0 * N * H * W * K * 9 * C
                x = (torch.randn((N, H, W, C), generator=g) * 0.5).to(bf).to(dev)
            ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=dev)
            dw = torch.empty((K, 3, 3, C), device=dev)
            dy = (torch.randn((N, H, W, K), generator=g) * 0.5).to(bf).to(dev)
            report(f"wgrad 3x3 {C}->{K} @{H}x{W}", flops,
                   lambda: call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, 3, 3, 1, 1, 1, H, W, ptr(dw), 0.0, 1,
                                ptr(ws), stream()), [dw])
            del ws, dw, dy
        else:
            report(f"fwd_dropout 3x3 {C}->{K} @64x128", flops,
                   lambda: call("acfe_conv2d_fwd_dropout", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b),
                                ptr(y), 1, ptr(st), 0.1, 5, stream()), [y])
        del x, y, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
