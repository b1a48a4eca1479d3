#!/usr/bin/env python3
"""How many steps do the Keras moving statistics (momentum 0.99) need to
settle?  Train test_learning_gpu's 4-class task for 300 steps (lr 1e-3), then
keep training at a small learning rate (the reference fit loop's
ReduceLROnPlateau cut) and classify the held-out clips through
Trainer.predict (eval mode, moving statistics, NO recalibration) after every
50 steps.  usage: python tools/learn_settle.py [fp32]"""
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
dtype = torch.float32 if "fp32" in sys.argv else torch.bfloat16
torch.manual_seed(0)
model = WRResNet(input_shape=(128, 513, 3), classes=4, dtype=dtype).to(dev)
fe = FrontEnd(n_mels=128, dtype=dtype, device=dev).to(dev)
tr = Trainer(model, fe, lr=1e-3, loss="cce", device=dev)
ops._seed_counter = itertools.count()
order = np.random.default_rng(3)
eye = torch.eye(4, device=dev)


def acc():
    pred = [tr.predict(xte[i:i + 64].contiguous()).float().argmax(1).cpu().numpy() for i in range(0, T.HELD, 64)]
    return float((np.concatenate(pred) == yte).mean())


def steps(n):
    ls = []
    for _ in range(n):
        idx = torch.from_numpy(order.choice(T.TRAIN, T.B, replace=False)).to(dev)
        loss, _ = tr.step(xtr[idx].contiguous(), eye[ytr[idx]])
        ls.append(float(loss))
    return np.mean(ls[-25:])


for k in range(6):
    l = steps(50)
    print(f"lr 1e-3 step {50 * (k + 1)}: loss {l:.4f} held-out acc (moving stats) {acc():.3f}", flush=True)
for lr in (1e-4, 1e-5):
    tr.opt.lr = lr
    for k in range(4):
        l = steps(50)
        print(f"lr {lr:g} +{50 * (k + 1)} steps: loss {l:.4f} held-out acc (moving stats) {acc():.3f}", flush=True)
