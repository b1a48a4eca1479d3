#!/usr/bin/env python3
"""Probe of the learning test's settings (tests/test_learning_gpu.py): loss
curves and held-out accuracy of wr_resnet_bird in bf16 / fp32 for a few
learning rates / step counts, eval with the moving statistics as trained and
after a momentum-0 recalibration pass.  usage: python tools/learn_probe.py"""
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
xte, yte = T.dataset(T.HELD, 2)
xtr, ytr, xte = torch.from_numpy(xtr).to(dev), torch.from_numpy(ytr).to(dev), torch.from_numpy(xte).to(dev)


def acc(tr):
    pred = []
    for i in range(0, T.HELD, 64):
        pred.append(tr.predict(xte[i:i + 64].contiguous()).float().argmax(1).cpu().numpy())
    p = np.concatenate(pred)
    return float((p == yte).mean()), np.bincount(p, minlength=4).tolist()


for lr, steps in [(1e-3, 300), (3e-3, 300), (1e-2, 300)]:
    for dtype in (torch.bfloat16, torch.float32):
        torch.manual_seed(0)
        model = WRResNet(input_shape=(128, 513, 3), classes=4, dtype=dtype).to(dev)
        fe = FrontEnd(n_mels=128, dtype=dtype, device=dev).to(dev)
        tr = Trainer(model, fe, lr=lr, loss="cce", device=dev)
        ops._seed_counter = itertools.count()
        order = np.random.default_rng(3)
        eye = torch.eye(4, device=dev)
        losses = []
        for _ in range(steps):
            idx = torch.from_numpy(order.choice(T.TRAIN, T.B, replace=False)).to(dev)
            loss, _ = tr.step(xtr[idx].contiguous(), eye[ytr[idx]])
            losses.append(float(loss))
        a0 = acc(tr)
        bns = [m for m in model.modules() if hasattr(m, "momentum") and hasattr(m, "moving_mean")]
        old = [m.momentum for m in bns]
        for m in bns:
            m.momentum = 0.0
        with torch.no_grad():
            model.train()
            model(fe(xtr[:128].contiguous()))
        for m, o in zip(bns, old):
            m.momentum = o
        a1 = acc(tr)
        w = [round(float(np.mean(losses[s - 25:s])), 3) for s in range(25, steps + 1, 25)]
        print(f"lr {lr} {str(dtype)[6:]} steps {steps}: acc moving {a0} recal {a1} loss25 {w}", flush=True)
