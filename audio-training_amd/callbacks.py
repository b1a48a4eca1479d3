"""The reference fit loop's callbacks (audiomodel.py:878-950) and validation
metrics (its compile(), :859-875), with Keras 3 semantics.

  checkpoints(run_dir, multi_label) -> the reference's list, in its order:
      ModelCheckpoint(save_best_only, weights only) for val_loss, val_precision,
      val_auc, val_recall, val_huber_loss, val_binary_focal_crossentropy and the
      accuracy (val_binary_accuracy / val_categorical_accuracy); mode "auto" for
      the losses, "max" for the rest (:893-906)
      EarlyStopping(patience=10, monitor="val_loss", mode="min") (:908-913)
      ReduceLROnPlateau(monitor="val_loss", mode="max") with Keras defaults
      factor 0.1, patience 10, min_delta 1e-4, cooldown 0, min_lr 0 (:914-917).
      mode="max" on a loss is the reference's own setting, reproduced as is:
      the LR is cut every 10 epochs while val_loss keeps FALLING.
      ModelCheckpoint("chkpt.weights.h5", save_freq="epoch") (:932-938).
  The TensorBoard / weight-histogram / EpochUpdater callbacks write logs only
  and are out of scope.

A callback sees `on_epoch_end(epoch, logs, fit)`, where `fit` exposes
`save(path)` (weights in the Keras *.weights.h5 layout), `lr` (read/write)
and `stop_training` -- the parts of keras.Model the reference's callbacks use.
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np

__all__ = ["ModelCheckpoint", "EarlyStopping", "ReduceLROnPlateau", "checkpoints", "ValMetrics"]


def _monitor_op(mode: str, monitor: str):
    """Keras ModelCheckpoint / EarlyStopping "auto": max for accuracy-like
    monitors ("acc" in the name, "fmeasure", "auc"), min otherwise."""
    if mode == "auto":
        low = monitor.lower()
        mode = "max" if ("acc" in low or low.startswith("fmeasure") or "auc" in low) else "min"
    return mode


class ModelCheckpoint:
    """keras.callbacks.ModelCheckpoint(filepath, monitor, save_best_only,
    save_weights_only=True, mode, save_freq="epoch")."""

    def __init__(self, filepath, monitor="val_loss", save_best_only=False, mode="auto"):
        self.filepath = Path(filepath)
        self.monitor, self.save_best_only = monitor, save_best_only
        self.mode = _monitor_op(mode, monitor)
        self.best = math.inf if self.mode == "min" else -math.inf
        self.saved_epochs: list[int] = []

    def on_epoch_end(self, epoch, logs, fit):
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None or (isinstance(cur, float) and math.isnan(cur)):
                return
            better = cur < self.best if self.mode == "min" else cur > self.best
            if not better:
                return
            self.best = cur
        fit.save(self.filepath)
        self.saved_epochs.append(epoch)


class EarlyStopping:
    """keras.callbacks.EarlyStopping(monitor, patience, mode, min_delta=0,
    baseline=None, restore_best_weights=False, start_from_epoch=0)."""

    def __init__(self, monitor="val_loss", patience=0, mode="auto", min_delta=0.0):
        self.monitor, self.patience = monitor, patience
        self.mode = _monitor_op(mode, monitor)
        self.min_delta = abs(min_delta) * (1 if self.mode == "max" else -1)
        self.best = math.inf if self.mode == "min" else -math.inf
        self.wait = 0
        self.best_epoch = 0
        self.stopped_epoch = 0

    def _improved(self, cur, ref):
        return (cur - self.min_delta < ref) if self.mode == "min" else (cur - self.min_delta > ref)

    def on_epoch_end(self, epoch, logs, fit):
        cur = logs.get(self.monitor)
        if cur is None:
            return
        self.wait += 1
        if self._improved(cur, self.best):
            self.best, self.best_epoch, self.wait = cur, epoch, 0
            return
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            fit.stop_training = True


class ReduceLROnPlateau:
    """keras.callbacks.ReduceLROnPlateau(monitor, factor=0.1, patience=10,
    mode, min_delta=1e-4, cooldown=0, min_lr=0.0)."""

    def __init__(self, monitor="val_loss", factor=0.1, patience=10, mode="auto", min_delta=1e-4, cooldown=0,
                 min_lr=0.0):
        if factor >= 1.0:
            raise ValueError("ReduceLROnPlateau does not support a factor >= 1.0")
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.min_delta, self.cooldown, self.min_lr = min_delta, cooldown, min_lr
        # Keras: "min", or "auto" without "acc" in the monitor, is the min mode
        self.mode = "min" if (mode == "min" or (mode == "auto" and "acc" not in monitor)) else "max"
        self.best = math.inf if self.mode == "min" else -math.inf
        self.cooldown_counter = 0
        self.wait = 0
        self.cut_epochs: list[int] = []

    def _better(self, cur, best):
        return cur < best - self.min_delta if self.mode == "min" else cur > best + self.min_delta

    def on_epoch_end(self, epoch, logs, fit):
        logs["learning_rate"] = float(fit.lr)
        cur = logs.get(self.monitor)
        if cur is None:
            return
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if self._better(cur, self.best):
            self.best, self.wait = cur, 0
        elif not self.cooldown_counter > 0:
            self.wait += 1
            if self.wait >= self.patience:
                old = float(fit.lr)
                if old > np.float32(self.min_lr):
                    fit.lr = max(old * self.factor, self.min_lr)
                    self.cut_epochs.append(epoch)
                    self.cooldown_counter = self.cooldown
                    self.wait = 0


def checkpoints(run_dir, multi_label=True):
    """AudioModel.checkpoints (audiomodel.py:878-950), the callbacks that act
    on training (in the reference's order)."""
    run_dir = Path(run_dir)
    metrics = ["val_loss", "val_precision", "val_auc", "val_recall", "val_huber_loss",
               "val_binary_focal_crossentropy", "val_binary_accuracy" if multi_label else "val_categorical_accuracy"]
    checks: list = []
    for m in metrics:
        mode = "auto" if ("loss" in m or "focal" in m) else "max"
        checks.append(ModelCheckpoint(run_dir / f"{m}.weights.h5", monitor=m, save_best_only=True, mode=mode))
    checks.append(EarlyStopping(patience=10, monitor="val_loss", mode="min"))
    checks.append(ReduceLROnPlateau(monitor="val_loss", mode="max"))
    checks.append(ModelCheckpoint(run_dir / "chkpt.weights.h5"))
    return checks


class ValMetrics:
    """The compile() metrics of audiomodel.py:859-875 over a validation pass,
    accumulated batch by batch as Keras' stateful metrics are: the model
    output is the activation (sigmoid multi-label, softmax single-label) of
    the logits.  Sums are kept as float64 device tensors so that data-parallel
    ranks add them with one all-reduce (`totals` / `from_totals`).

      accuracy: binary (p > 0.5 == y) or categorical (argmax match)
      precision / recall: thresholds 0.5 over every (clip, class) element
      auc: ROC, 200 thresholds, interpolated (Keras AUC defaults)
      huber_loss: delta 1 on (y, p), mean over classes, then clips
      binary_focal_crossentropy: gamma 2, no class balancing, mean over classes
    """

    NT = 200

    def __init__(self, multi_label, device):
        import torch

        self.multi_label = multi_label
        eps = 1e-7
        th = [(i + 1) / (self.NT - 1) for i in range(self.NT - 2)]
        self.thresholds = torch.tensor([0.0 - eps] + th + [1.0 + eps], dtype=torch.float32, device=device)
        # [loss sum, correct, n, tp, fp, fn, huber sum, focal sum] + 4 x NT AUC counts
        self.sums = torch.zeros(8 + 4 * self.NT, dtype=torch.float64, device=device)

    def update(self, z, y, loss):
        import torch

        z, y = z.float(), y.float()
        p = torch.sigmoid(z) if self.multi_label else torch.softmax(z, dim=1)
        b = z.shape[0]
        if self.multi_label:
            correct = ((p > 0.5).float() == y).float().mean(1).sum()
        else:
            correct = (p.argmax(1) == y.argmax(1)).float().sum()
        pred = (p > 0.5).float()
        tp, fp, fn = (pred * y).sum(), (pred * (1 - y)).sum(), ((1 - pred) * y).sum()
        d = (y - p).abs()
        huber = torch.where(d <= 1.0, 0.5 * d * d, d - 0.5).mean(1).sum()
        pc = p.clamp(1e-7, 1 - 1e-7)
        bce = -(y * torch.log(pc) + (1 - y) * torch.log(1 - pc))
        pt = y * pc + (1 - y) * (1 - pc)
        focal = ((1 - pt) ** 2 * bce).mean(1).sum()
        gt = (p.reshape(-1, 1) > self.thresholds.reshape(1, -1)).float()  # [elements, NT]
        yf = y.reshape(-1, 1)
        a_tp, a_fp = (gt * yf).sum(0), (gt * (1 - yf)).sum(0)
        a_fn, a_tn = ((1 - gt) * yf).sum(0), ((1 - gt) * (1 - yf)).sum(0)
        head = torch.stack([loss.double().sum() * b, correct.double(), torch.tensor(float(b), device=z.device,
                                                                                     dtype=torch.float64),
                            tp.double(), fp.double(), fn.double(), huber.double(), focal.double()])
        self.sums += torch.cat([head, a_tp.double(), a_fp.double(), a_fn.double(), a_tn.double()])

    def totals(self):
        return self.sums

    def result(self, sums=None):
        s = (self.sums if sums is None else sums).double().cpu().numpy()
        n = s[2]
        if not n:
            return {}
        tp, fp, fn = s[3], s[4], s[5]
        a = s[8:].reshape(4, self.NT)
        tpr = np.divide(a[0], a[0] + a[2], out=np.zeros(self.NT), where=(a[0] + a[2]) > 0)
        fpr = np.divide(a[1], a[1] + a[3], out=np.zeros(self.NT), where=(a[1] + a[3]) > 0)
        auc = float(np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2.0))
        acc = "val_binary_accuracy" if self.multi_label else "val_categorical_accuracy"
        return {"val_loss": s[0] / n, acc: s[1] / n,
                "val_precision": tp / (tp + fp) if tp + fp > 0 else 0.0,
                "val_recall": tp / (tp + fn) if tp + fn > 0 else 0.0,
                "val_auc": auc, "val_huber_loss": s[6] / n, "val_binary_focal_crossentropy": s[7] / n}
