#!/usr/bin/env python3
"""After N training steps: each BatchNormalization's moving mean / variance
against the batch statistics of one more training-mode forward (momentum-0
recalibration) -- are the moving statistics tracking?  usage: python tools/bn_moving_probe.py"""
import itertools
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_learning_gpu as T  # noqa: E402
from acfe import ops  # noqa: E402
from acfe.train import FrontEnd, Trainer  # noqa: E402
from resnet.wr_resnet_bird import WRResNet  # noqa: E402

dev = torch.device("cuda", 0)
xtr, ytr = T.dataset(T.TRAIN, 1)
xtr, ytr = torch.from_numpy(xtr).to(dev), torch.from_numpy(ytr).to(dev)
dtype = torch.float32 if "fp32" in sys.argv else torch.bfloat16
steps = 300
torch.manual_seed(0)
model = WRResNet(input_shape=(128, 513, 3), classes=4, dtype=dtype).to(dev)
fe = FrontEnd(n_mels=128, dtype=dtype, device=dev).to(dev)
tr = Trainer(model, fe, lr=1e-3, loss="cce", device=dev)
ops._seed_counter = itertools.count()
order = np.random.default_rng(3)
eye = torch.eye(4, device=dev)
bns = [(n, m) for n, m in model.named_modules() if hasattr(m, "moving_mean")]
init = {n: (m.moving_mean.clone(), m.moving_variance.clone()) for n, m in bns}
for i in range(steps):
    idx = torch.from_numpy(order.choice(T.TRAIN, T.B, replace=False)).to(dev)
    tr.step(xtr[idx].contiguous(), eye[ytr[idx]])
before = {n: (m.moving_mean.clone(), m.moving_variance.clone()) for n, m in bns}
for _, m in bns:
    m.momentum = 0.0
with torch.no_grad():
    model.train()
    model(fe(xtr[:128].contiguous()))
for n, m in bns:
    mm0, mv0 = init[n]
    mm, mv = before[n]
    bm, bv = m.moving_mean, m.moving_variance
    moved = float((mm - mm0).abs().max())
    dm = float((mm - bm).abs().max() / (bv.sqrt().max() + 1e-6))
    dv = float(((mv - bv).abs() / (bv + 1e-6)).max())
    print(f"{n:40s} moved {moved:9.3e}  |mean-batch|/std {dm:8.3f}  |var-batch|/var {dv:8.3f}", flush=True)
