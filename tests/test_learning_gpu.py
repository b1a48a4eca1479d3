"""The device training step learns, in bf16 and fp32.

A synthetic 4-class task in which each class is a chirp in its own frequency
band (build.synth_clip's generator restricted to one band per class, at a
random gain, onset and duration over noise).  wr_resnet_bird (the T1 model,
resnet/wr_resnet_bird.py) trains through acfe.train.Trainer -- raw clips ->
normalize -> STFT / mel -> PCEN -> model -> CCE -> backward -> Keras Adam,
the reference fit loop's step (audiomodel.py:550-562, loss / optimizer
:1206-1240) -- with mix_up off, from the same initial weights in bf16 (T1's
precision) and fp32 (the reference default).  Held-out clips are classified by
Trainer.predict (eval-mode BN).  This is the behavioural check that the whole
bf16 training-mode path (every BN backward, dropout, the fused nodes) moves the
model the way fp32 does, which the per-block tests cannot show.

Evaluation: Keras's moving statistics (momentum 0.99) still lag the weights
after a few hundred steps (tools/bn_moving_probe.py, tools/learn_probe.py:
held-out accuracy at chance with them, 99-100 % with current statistics), so
before predicting, one training-mode forward over 128 training clips with
momentum 0 sets every BatchNormalization's moving statistics to the current
batch statistics ("BN recalibration"; the reference fit loop instead runs many
epochs).

Bounds: held-out accuracy >= 90 % for both; the bf16 loss, averaged over each
25-step window, within LOSS_BAND of the fp32 one in the same window or a
neighbouring one.  When each run leaves the ln(4) plateau is chaotic (any
change of summation order moves it by tens of steps: 0.27 apart at worst in the
probe, 0.48 in r05q when the fp32 convolutions' K-tile order changed, with the
bf16 curve one window behind), so the curves are compared up to a 25-step
shift, not step for step.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SR = 48000
N = 3 * SR
BANDS = [(600.0, 1400.0), (1800.0, 3200.0), (4000.0, 6000.0), (7000.0, 10500.0)]
B, STEPS, TRAIN, HELD = 32, 300, 512, 128
LOSS_BAND = 0.4  # |mean bf16 loss - mean fp32 loss| over each 25-step window


def band_clip(rng, k):
    t = np.arange(N) / SR
    x = rng.normal(0, rng.uniform(0.002, 0.02), N)
    lo, hi = BANDS[k]
    for _ in range(rng.integers(1, 3)):
        f0, f1 = rng.uniform(lo, hi, 2)
        amp, on = rng.uniform(0.05, 0.5), rng.uniform(0, 1.5)
        dur = rng.uniform(0.5, 3.0 - on)
        m = (t >= on) & (t < on + dur)
        tt = t[m] - on
        x[m] += amp * np.sin(2 * np.pi * (f0 * tt + 0.5 * (f1 - f0) / dur * tt * tt))
    return np.clip(x, -1, 1).astype(np.float32)


def dataset(n, seed):
    rng = np.random.default_rng(seed)
    labels = np.arange(n) % len(BANDS)
    rng.shuffle(labels)
    return np.stack([band_clip(rng, int(k)) for k in labels]), labels


@pytest.fixture(scope="module")
def data(cuda):
    xtr, ytr = dataset(TRAIN, 1)
    xte, yte = dataset(HELD, 2)
    return (torch.from_numpy(xtr).to(cuda), torch.from_numpy(ytr).to(cuda),
            torch.from_numpy(xte).to(cuda), yte)


def train(dtype, data, cuda):
    from acfe import ops
    from acfe.train import FrontEnd, Trainer
    from resnet.wr_resnet_bird import WRResNet
    import itertools

    xtr, ytr, xte, yte = data
    torch.manual_seed(0)
    model = WRResNet(input_shape=(128, 513, 3), classes=len(BANDS), dtype=dtype).to(cuda)
    fe = FrontEnd(n_mels=128, dtype=dtype, device=cuda).to(cuda)
    tr = Trainer(model, fe, lr=1e-3, loss="cce", device=cuda)
    ops._seed_counter = itertools.count()
    order = np.random.default_rng(3)
    losses = []
    eye = torch.eye(len(BANDS), device=cuda)
    for _ in range(STEPS):
        idx = torch.from_numpy(order.choice(TRAIN, B, replace=False)).to(cuda)
        loss, _ = tr.step(xtr[idx].contiguous(), eye[ytr[idx]])
        losses.append(float(loss))
    torch.cuda.synchronize()
    bns = [m for m in model.modules() if hasattr(m, "moving_mean")]
    for m in bns:
        m.momentum, m._m = 0.0, m.momentum
    with torch.no_grad():
        model.train()
        model(fe(xtr[:128].contiguous()))
    for m in bns:
        m.momentum = m._m
    pred = []
    for i in range(0, HELD, 64):
        pred.append(tr.predict(xte[i:i + 64].contiguous()).float().argmax(1).cpu().numpy())
    acc = float((np.concatenate(pred) == yte).mean())
    return np.array(losses), acc


def test_training_learns_bf16_and_fp32(data, cuda):
    l16, a16 = train(torch.bfloat16, data, cuda)
    l32, a32 = train(torch.float32, data, cuda)
    w16 = [l16[s - 25:s].mean() for s in range(25, STEPS + 1, 25)]
    w32 = [l32[s - 25:s].mean() for s in range(25, STEPS + 1, 25)]
    print("loss bf16", np.round(w16, 4), "acc", a16)
    print("loss fp32", np.round(w32, 4), "acc", a32)
    assert np.isfinite(l16).all() and np.isfinite(l32).all()
    assert w32[-1] < 0.2 * w32[0] and w16[-1] < 0.2 * w16[0]
    assert a32 >= 0.9 and a16 >= 0.9, (a16, a32)
    for i, a in enumerate(w16):
        near = w32[max(i - 1, 0):i + 2]
        assert min(abs(a - b) for b in near) <= LOSS_BAND, (i, w16, w32)
