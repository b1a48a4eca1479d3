"""The reference fit loop's callbacks (audiomodel.py:878-950) on synthetic
val_loss sequences, CPU only: which epochs cut the learning rate, which epoch
stops training, which epochs write which checkpoint.  Keras semantics are
restated (Keras is not importable here): EarlyStopping / ReduceLROnPlateau /
ModelCheckpoint of Keras 3 with the reference's arguments.  ValMetrics
against numpy / scikit-learn on random predictions."""
import math
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-training_amd"))

import callbacks  # noqa: E402


class FakeFit:
    def __init__(self, lr=0.01):
        self.lr = lr
        self.stop_training = False
        self.saved = []

    def save(self, path):
        self.saved.append(Path(path).name)


def run(seq, multi_label=False, extra=None):
    """Drive the reference's callbacks over val_loss values `seq` (and other
    val_* logs from `extra(epoch)`) until EarlyStopping stops the loop."""
    checks = callbacks.checkpoints("/nonexistent/run", multi_label=multi_label)
    fit = FakeFit()
    lrs, saves = [], []
    for epoch, v in enumerate(seq):
        logs = {"loss": v, "val_loss": v}
        if extra is not None:
            logs.update(extra(epoch))
        fit.saved = []
        for cb in checks:
            cb.on_epoch_end(epoch, logs, fit)
        lrs.append(fit.lr)
        saves.append(list(fit.saved))
        if fit.stop_training:
            break
    return checks, lrs, saves


def test_reference_callback_list():
    checks = callbacks.checkpoints("/r", multi_label=False)
    names = [type(c).__name__ for c in checks]
    assert names == ["ModelCheckpoint"] * 7 + ["EarlyStopping", "ReduceLROnPlateau", "ModelCheckpoint"]
    mons = [c.monitor for c in checks[:7]]
    assert mons == ["val_loss", "val_precision", "val_auc", "val_recall", "val_huber_loss",
                    "val_binary_focal_crossentropy", "val_categorical_accuracy"]
    # "auto" on the losses resolves to min, "max" for the rest (audiomodel.py:895-898)
    assert [c.mode for c in checks[:7]] == ["min", "max", "max", "max", "min", "min", "max"]
    assert callbacks.checkpoints("/r", multi_label=True)[6].monitor == "val_binary_accuracy"
    es, rl, ck = checks[7], checks[8], checks[9]
    assert (es.monitor, es.patience, es.mode) == ("val_loss", 10, "min")
    assert (rl.monitor, rl.mode, rl.factor, rl.patience, rl.min_delta) == ("val_loss", "max", 0.1, 10, 1e-4)
    assert ck.filepath.name == "chkpt.weights.h5" and not ck.save_best_only


def test_falling_val_loss_cuts_lr_every_ten_epochs():
    """mode="max" on val_loss (the reference's setting): while val_loss falls
    nothing counts as an improvement after epoch 0, so the LR drops x0.1 at
    epochs 10, 20 and 30; EarlyStopping (mode min) never fires."""
    seq = [1.0 - 0.01 * e for e in range(35)]
    checks, lrs, saves = run(seq)
    rl = checks[8]
    assert rl.cut_epochs == [10, 20, 30]
    exp = [0.01 * 0.1 ** sum(e >= c for c in (10, 20, 30)) for e in range(35)]
    np.testing.assert_allclose(lrs, exp, rtol=1e-12)
    assert len(lrs) == 35 and not checks[7].stopped_epoch
    # best val_loss improves every epoch: its checkpoint and chkpt every epoch
    assert all("val_loss.weights.h5" in s and "chkpt.weights.h5" in s for s in saves)


def test_plateau_stops_after_patience():
    """val_loss falls for 5 epochs (best at epoch 4), then stays above it:
    EarlyStopping stops at epoch 4 + 10 = 14; the LR was cut once, at epoch
    10 (ten non-improving epochs in mode max since epoch 0)."""
    seq = [1.0, 0.9, 0.8, 0.7, 0.6] + [0.65] * 20
    checks, lrs, saves = run(seq)
    es, rl = checks[7], checks[8]
    assert es.stopped_epoch == 14 and es.best_epoch == 4 and len(lrs) == 15
    assert rl.cut_epochs == [10]
    assert lrs[9] == pytest.approx(0.01) and lrs[10] == pytest.approx(0.001)
    assert [e for e, s in enumerate(saves) if "val_loss.weights.h5" in s] == [0, 1, 2, 3, 4]


def test_rising_val_loss_resets_lr_wait():
    """In mode max a RISING val_loss (by more than min_delta) is an
    improvement: it resets the plateau counter."""
    seq = [1.0, 0.9, 0.8, 0.7, 0.6, 0.5, 0.4, 0.3, 0.2, 1.5, 0.1, 0.09, 0.08]
    checks, lrs, _ = run(seq)
    assert checks[8].cut_epochs == []  # epoch 9 reset the counter before it reached 10
    assert checks[7].stopped_epoch == 0  # val_loss kept improving overall


def test_metric_checkpoints_modes():
    """The max-mode metric checkpoints save on increases only."""
    prec = [0.5, 0.6, 0.55, 0.7, 0.7]
    _, _, saves = run([1.0] * 5, extra=lambda e: {"val_precision": prec[e]})
    assert [e for e, s in enumerate(saves) if "val_precision.weights.h5" in s] == [0, 1, 3]


def test_val_metrics_against_numpy():
    from sklearn.metrics import roc_auc_score

    g = torch.Generator().manual_seed(5)
    B, C = 64, 6
    vm = callbacks.ValMetrics(True, "cpu")
    zs, ys = [], []
    for _ in range(3):
        z = torch.randn((B, C), generator=g) * 2
        y = (torch.rand((B, C), generator=g) < 0.3).float()
        zs.append(z)
        ys.append(y)
        vm.update(z, y, torch.tensor(0.5))
    r = vm.result()
    z, y = torch.cat(zs).numpy().astype(np.float64), torch.cat(ys).numpy()
    p = 1 / (1 + np.exp(-z))
    pred = p > 0.5
    tp, fp, fn = (pred & (y > 0)).sum(), (pred & (y == 0)).sum(), (~pred & (y > 0)).sum()
    assert r["val_precision"] == pytest.approx(tp / (tp + fp), rel=1e-9)
    assert r["val_recall"] == pytest.approx(tp / (tp + fn), rel=1e-9)
    assert r["val_binary_accuracy"] == pytest.approx((pred == (y > 0)).mean(), rel=1e-6)  # f32 row means
    # Keras AUC: 200 thresholds, interpolated -- within 5e-3 of the exact ROC AUC
    assert abs(r["val_auc"] - roc_auc_score(y.reshape(-1), p.reshape(-1))) < 5e-3
    d = np.abs(y - p)
    assert r["val_huber_loss"] == pytest.approx(np.where(d <= 1, 0.5 * d * d, d - 0.5).mean(), rel=1e-5)
    pc = np.clip(p, 1e-7, 1 - 1e-7)
    bce = -(y * np.log(pc) + (1 - y) * np.log(1 - pc))
    pt = y * pc + (1 - y) * (1 - pc)
    assert r["val_binary_focal_crossentropy"] == pytest.approx(((1 - pt) ** 2 * bce).mean(), rel=1e-5)
    assert r["val_loss"] == pytest.approx(0.5)
    assert math.isfinite(r["val_auc"])
