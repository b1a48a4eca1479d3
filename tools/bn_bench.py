#!/usr/bin/env python3
"""Bandwidth of the BatchNormalization passes on a stage-1 tensor of the T1
step ([512, 64, 128, C] bf16): acfe_bn_apply (+ReLU), acfe_bn_bwd_reduce and
acfe_bn_bwd_apply_ex in the variants the model uses (plain, + residual add,
+ dropout, with / without the fused channel sums of dx), HIP events on the
launch stream.  usage: python tools/bn_bench.py [--C 64] [--iters 9]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402


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
    ap.add_argument("--C", type=int, default=64)
    ap.add_argument("--iters", type=int, default=9)
    a = ap.parse_args()
    from acfe._lib import call, lib
    from acfe._torch import ptr, stream

    dev = torch.device("cuda", 0)
    N, H, W, C = 512, 64, 128, a.C
    rows = N * H * W
    n = rows * C
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(dev)
    dy = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(dev)
    add = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(dev)
    out = torch.empty_like(x)
    sc, sh, mu, iv = (torch.rand(C, device=dev) + 0.5 for _ in range(4))
    coef = torch.rand(3 * C, device=dev)
    nr = lib.acfe_reduce_blocks(rows)
    part = torch.empty((nr, 2, C), dtype=torch.float64, device=dev)
    sums = torch.empty((nr, 2, C), dtype=torch.float64, device=dev)

    def rep(name, nbytes, fn):
        t = timeit(fn, a.iters)
        print(f"{name:44s} {t * 1e3:8.1f} us  {nbytes / t / 1e9:6.2f} TB/s", flush=True)

    rep("bn_apply relu (2+2 B/elem)", 4 * n,
        lambda: call("acfe_bn_apply", ptr(x), 1, rows, C, ptr(sc), ptr(sh), 1, ptr(out), 1, stream()))
    rep("bn_bwd_reduce relu (2+2 B/elem)", 4 * n,
        lambda: call("acfe_bn_bwd_reduce", ptr(dy), 1, ptr(x), 1, rows, C, ptr(sc), ptr(sh), ptr(mu), ptr(iv), 1,
                     ptr(part), stream()))
    for nm, ad, rate, sm in (("plain", None, 0.0, None), ("plain+sums", None, 0.0, sums),
                             ("add", add, 0.0, None), ("add+sums", add, 0.0, sums),
                             ("dropout", None, 0.1, None), ("dropout+sums", None, 0.1, sums)):
        nb = (8 if ad is not None else 6) * n
        rep(f"bn_bwd_apply {nm} ({nb // n} B/elem)", nb,
            lambda ad=ad, rate=rate, sm=sm: call("acfe_bn_bwd_apply_ex", ptr(dy), 1, ptr(x), 1, rows, C, ptr(sc),
                                                 ptr(sh), 1, ptr(coef), ptr(ad), rate, 11, ptr(out), 1, ptr(sm),
                                                 stream()))
    rep("torch copy (2+2 B/elem)", 4 * n, lambda: out.copy_(x))


if __name__ == "__main__":
    main()
