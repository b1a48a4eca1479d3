#!/usr/bin/env python3
"""Per-layer conv timing of one T1 training step (wr_resnet_bird, batch 512,
bf16): HIP events around every conv's fwd / dgrad / wgrad (ops.watch_conv),
with the layer's shape and achieved TFLOP/s.
usage: python tools/layer_profile.py [batch] [wrn]   (wrn: wr_resnet, 2 classes)"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import numpy as np
import torch
import bench
from acfe import ops
from acfe.train import FrontEnd, Trainer

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
WRN = len(sys.argv) > 2 and sys.argv[2] == "wrn"
if WRN:
    from resnet.wr_resnet import WRResNet
else:
    from resnet.wr_resnet_bird import WRResNet
NCLS = 2 if WRN else 50
model = WRResNet(input_shape=(128, 513, 3), classes=NCLS, dtype=torch.bfloat16).to(dev)
fe = FrontEnd(n_mels=128, dtype=torch.bfloat16, device=dev).to(dev)
tr = Trainer(model, fe, lr=0.01, loss="cce", device=dev)
x1, x2, lam, y = bench.make_batches(B, NCLS, dev, n_sets=1)[0]
for _ in range(2):
    tr.step(x1, y, x2, lam)
torch.cuda.synchronize()
convs = [(n, m) for n, m in model.named_modules() if hasattr(m, "weight") and m.weight is not None and m.weight.dim() == 4]
stores = {}
for n, m in convs:
    stores[n] = []
    ops.watch_conv(m.weight, stores[n])
shapes = {}
hooks = [m.register_forward_pre_hook(lambda mod, inp, n=n: shapes.__setitem__(n, tuple(inp[0].shape))) for n, m in convs]
tr.step(x1, y, x2, lam)
torch.cuda.synchronize()
tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
print(f"{'layer':40s} {'in NHWC':22s} {'K R S':10s} {'fwd ms':>8s} {'dgrad':>8s} {'wgrad':>8s}  TF(f/d/w)")
for n, m in convs:
    K, R, S, C = m.weight.shape
    d = {k: sum(e0.elapsed_time(e1) for kk, e0, e1 in stores[n] if kk == k) for k in tot}
    for k in tot:
        tot[k] += d[k]
    shp = shapes.get(n, ())
    if len(shp) == 4:
        N_, H, W, C_ = shp
    else:
        N_, H, W, C_ = (B, 0, 0, C)
    fl = 2.0 * N_ * H * W * K * R * S * C  # stride-1 "same" approximation
    tf = [fl / (d[k] * 1e-3) / 1e12 if d[k] > 0 else 0 for k in ("fwd", "dgrad", "wgrad")]
    print(f"{n:40s} {str(shp):22s} {f'{K} {R}x{S}':10s} {d['fwd']:8.3f} {d['dgrad']:8.3f} {d['wgrad']:8.3f}  "
          f"{tf[0]:.0f}/{tf[1]:.0f}/{tf[2]:.0f}")
print(f"total conv ms: fwd {tot['fwd']:.2f} dgrad {tot['dgrad']:.2f} wgrad {tot['wgrad']:.2f}")
