#!/usr/bin/env python3
"""Training driver of the acfe path (reference audiomodel.py:117-567, CLI :2238-2414).

  python audiomodel.py RUN_NAME -d DATA_DIR [--model-name wr-resnet-bird|wr-resnet]
         [--epochs E] [--batch-size B] [--n_mels 128] [--multi-label false] [--lr 0.01]
  multi-GPU:  python -m torch.distributed.run --nproc-per-node 8 audiomodel.py ...

DATA_DIR is the directory holding training-data/ (build.py output):
training-meta.json gives the labels; train/ and validation/ hold the GZIP
TFRecord shards.  The reference flow (load_datasets -> build_model -> compile
-> fit with checkpoints -> save metadata) becomes: tfdataset.get_dataset
(raw audio batches, mix_up pairs when augmenting) -> acfe.train.FrontEnd (GPU
normalize / mix_up / STFT / mel / PCEN) + resnet WRResNet -> acfe.train.Trainer
(loss, backward, RCCL all-reduce, Adam) -> checkpoints/<run>/ {model.pt,
metadata.txt}.  Dataset curation options of the reference (taxonomy remaps,
cross-fold, rf/embeddings models) are out of scope.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

import torch  # noqa: E402


def str2bool(v):
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("yes", "true", "t", "y", "1")


MODEL_NAMES = {"wr-resnet": "wr_resnet", "wr-resnet-bird": "wr_resnet_bird", "wr_resnet": "wr_resnet",
               "wr_resnet_bird": "wr_resnet_bird"}


def build_model(model_name, input_shape, classes, dtype, dropout=0.1):
    """AudioModel.build_model for the wr-resnet branches (audiomodel.py:776-780)."""
    kind = MODEL_NAMES[model_name]
    if kind == "wr_resnet_bird":
        from resnet.wr_resnet_bird import WRResNet
    else:
        from resnet.wr_resnet import WRResNet
    return WRResNet(input_shape=input_shape, classes=classes, dtype=dtype, dropout=dropout)


def load_meta(data_dir):
    base = Path(data_dir)
    for cand in (base / "training-meta.json", base / "training-data" / "training-meta.json"):
        if cand.exists():
            return json.loads(cand.read_text()), cand.parent
    raise FileNotFoundError(f"training-meta.json not found under {data_dir}")


def save_checkpoint(out_dir: Path, trainer, meta: dict, history: dict | None = None):
    """model.pt (front end + model state) and the model's weights in the Keras 3
    `*.weights.h5` layout the reference's checkpoints use (audiomodel.py:878-938)."""
    from keras_weights import save_keras_weights

    out_dir.mkdir(parents=True, exist_ok=True)
    torch.save({k: v.detach().cpu() for k, v in trainer.holder.state_dict().items()}, out_dir / "model.pt")
    save_keras_weights(trainer.model, out_dir / "model.weights.h5")
    m = dict(meta)
    if history:
        m["history"] = history
    (out_dir / "metadata.txt").write_text(json.dumps(m, indent=2))


def evaluate(trainer, dataset, multi_label, group=None):
    """The validation pass of model.fit (audiomodel.py:550-562): the compiled
    metrics of :859-875 (callbacks.ValMetrics: loss, accuracy, precision,
    recall, AUC, Huber, binary focal cross-entropy) as Keras names them
    (`val_*`).  Under data parallelism every rank evaluates its own shard and
    the metric sums are added over ranks with one all-reduce."""
    from acfe import dp, ops
    from callbacks import ValMetrics

    trainer.holder.eval()
    dev = trainer.device
    vm = ValMetrics(multi_label, dev)
    with torch.no_grad():
        for x, y in dp.synced_batches(dataset, group=group):
            f = trainer.frontend.forward_spec(x) if x.dim() == 3 else trainer.frontend(x)
            z = trainer.model(f)
            loss, _ = ops.loss_and_grad(z, y, trainer.loss_mode)
            vm.update(z, y, loss)
    trainer.holder.train()
    logs = vm.result(torch.tensor(dp.allreduce_sums(vm.totals().tolist(), device=dev), dtype=torch.float64))
    return logs or {"val_loss": float("nan")}


class _Fit:
    """What the reference's callbacks touch of keras.Model during fit: the
    optimizer's learning rate, stop_training, and save_weights (rank 0 writes,
    Keras *.weights.h5 layout)."""

    def __init__(self, trainer, rank):
        self.trainer, self.rank = trainer, rank
        self.stop_training = False

    @property
    def lr(self):
        return self.trainer.opt.lr

    @lr.setter
    def lr(self, v):
        self.trainer.opt.lr = float(v)

    def save(self, path):
        if self.rank == 0:
            from keras_weights import save_keras_weights

            Path(path).parent.mkdir(parents=True, exist_ok=True)
            save_keras_weights(self.trainer.model, path)


def train_epoch(dataset, step_fn, augment, steps_per_epoch=0, mixup_fn=None, group=None):
    """One pass of the fit loop (audiomodel.py:550-562) over `dataset`.
    step_fn(x1, y1, x2, y2, lam) -> device loss.  Every rank runs the same
    number of steps (acfe.dp.synced_batches over the host control group), and
    the loss is summed on the device and read once per epoch, not per step.
    Returns (clips, loss sum, steps) of this rank."""
    from acfe import dp

    lsum = None
    n = steps = 0
    for item in dp.synced_batches(dataset, group=group):
        if augment:
            (x1, y1), (x2, y2) = item
            loss = step_fn(x1, y1, x2, y2, mixup_fn(x1.shape[0]))
        else:
            x1, y1 = item
            loss = step_fn(x1, y1, None, None, None)
        contrib = loss.detach().double().sum() * x1.shape[0]
        lsum = contrib if lsum is None else lsum + contrib
        n += x1.shape[0]
        steps += 1
        if steps_per_epoch and steps >= steps_per_epoch:
            break
    return n, (float(lsum) if lsum is not None else 0.0), steps


def shard_files(files, rank, world):
    """Data-parallel input split: whole shard files per rank when there are at
    least as many files as ranks, else every rank reads all files and keeps its
    share of the records (AudioDataset record_shard)."""
    if world == 1:
        return list(files), None
    if len(files) >= world:
        return list(files)[rank::world], None
    return list(files), (rank, world)


def train_model(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import tfdataset
    from acfe import dp, ops
    from acfe.frontend import sample_mixup_lambda
    from acfe.train import FrontEnd, Trainer, mix_labels

    ctrl = dp.control_group()
    ops.set_seed_rank(rank)  # per-replica dropout masks
    meta, td = load_meta(args.dataset_dir)
    labels = list(meta["labels"])
    n_mels = args.n_mels or meta.get("n_mels", 160)
    fmin = args.fmin if args.fmin is not None else 100
    fmax = args.fmax if args.fmax is not None else 11000
    n_fft = args.n_fft or 4096
    brk = args.break_freq or 1000
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(args.seed)
    model = build_model(args.model_name, (n_mels, 513, 3), len(labels), dtype).to(dev)
    if world > 1:
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, 0)
    torch.manual_seed(args.seed + rank)  # per-replica mix_up lambdas after the shared init
    frontend = FrontEnd(n_mels=n_mels, n_fft=n_fft, hop=281, fmin=fmin, fmax=fmax, break_freq=brk,
                        pcen=args.pcen, dtype=dtype, device=dev).to(dev)
    trainer = Trainer(model, frontend, lr=args.lr, loss="bce" if args.multi_label else "cce", device=dev)
    if args.weights:
        if str(args.weights).endswith((".h5", ".keras")):  # reference checkpoints (audiomodel.py:569-595)
            from keras_weights import load_keras_weights

            load_keras_weights(model, args.weights)
        else:
            sd = torch.load(args.weights, map_location="cpu", weights_only=True)
            trainer.holder.load_state_dict(sd)
    files, rshard = shard_files(tfdataset._files(td / "train"), rank, world)
    load_raw = bool(args.load_raw)
    # tfdataset.get_dataset (audiomodel.py:1607-1621): this rank's share of the
    # shards; epoch_size = the examples one epoch of this rank yields
    train_ds, _, epoch_size, _, _ = tfdataset.get_dataset(
        td / "train", labels, files=files, record_shard=rshard, batch_size=args.batch_size, shuffle=args.shuffle,
        augment=args.augment and load_raw, device=dev, drop_remainder=world > 1, seed=args.seed, load_raw=load_raw)
    logging.info("rank %d: %d training examples, %d batches per epoch", rank, epoch_size, len(train_ds))
    val_dir = td / "validation"
    val_ds = None
    if val_dir.exists() and tfdataset._files(val_dir):
        vfiles, vshard = shard_files(tfdataset._files(val_dir), rank, world)
        val_ds, _, _, _, _ = tfdataset.get_dataset(val_dir, labels, files=vfiles, record_shard=vshard,
                                                   batch_size=args.batch_size, shuffle=False, device=dev,
                                                   load_raw=load_raw)
    history = {"loss": [], "val_loss": [], "val_accuracy": [], "clips_per_s": [], "learning_rate": []}
    out_dir = Path(args.checkpoint_dir) / args.name
    import callbacks

    # AudioModel.checkpoints (audiomodel.py:878-950): best-metric checkpoints,
    # EarlyStopping(10), ReduceLROnPlateau(val_loss, mode "max"), chkpt per epoch
    checks = callbacks.checkpoints(out_dir, multi_label=args.multi_label)
    fit = _Fit(trainer, rank)

    def step(x1, y1, x2, y2, lam):
        if x2 is None:
            return trainer.step(x1, y1)[0]
        return trainer.step(x1, mix_labels(y1, y2, lam), x2, lam)[0]

    def mixup(b):
        return sample_mixup_lambda(b, 0.5, 0.25, device=dev)

    for epoch in range(args.epochs):
        t0 = time.perf_counter()
        n, lsum, steps = train_epoch(train_ds, step, args.augment and load_raw, args.steps_per_epoch, mixup, ctrl)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n_all, lsum_all = dp.allreduce_sums([n, lsum], device=dev)
        logs = {"loss": lsum_all / max(n_all, 1)}
        history["loss"].append(logs["loss"])
        history["clips_per_s"].append(n_all / dt)
        # Keras SyncOnRead MEAN of the BN moving statistics before eval / save
        dp.average_buffers(trainer.holder)
        if val_ds is not None:
            logs.update(evaluate(trainer, val_ds, args.multi_label, ctrl))
            history["val_loss"].append(logs["val_loss"])
            history["val_accuracy"].append(logs.get("val_binary_accuracy", logs.get("val_categorical_accuracy")))
            for k, v in logs.items():
                if k.startswith("val_") and k not in ("val_loss",):
                    history.setdefault(k, []).append(v)
        for cb in checks:
            cb.on_epoch_end(epoch, logs, fit)
        history["learning_rate"].append(logs.get("learning_rate", fit.lr))
        if rank == 0:
            logging.info("epoch %d loss %.4f val %s lr %g %.1f clips/s (%d steps/rank)", epoch, history["loss"][-1],
                         history["val_loss"][-1:] or "-", fit.lr, history["clips_per_s"][-1], steps)
        if fit.stop_training:  # EarlyStopping
            break
    if rank == 0:
        meta_out = dict(meta)
        meta_out.update(name=args.model_name, ebird_labels=labels, labels=labels, n_mels=n_mels, fmin=fmin,
                        fmax=fmax, n_fft=n_fft, break_freq=brk, hop_length=281, power=2 if load_raw else 1, pcen=args.pcen,
                        multi_label=args.multi_label, loss_fn="bce" if args.multi_label else "cce", load_raw=load_raw,
                        dtype=args.dtype, training_date=str(time.time()), magv2=True)
        save_checkpoint(out_dir, trainer, meta_out, history)
        print(json.dumps({"run": args.name, "epochs": len(history["loss"]), "final_loss": history["loss"][-1],
                          "val_loss": history["val_loss"][-1:] or None, "clips_per_s": history["clips_per_s"]}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return history


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("name", help="Run name")
    p.add_argument("-d", "--dataset-dir", required=True)
    p.add_argument("--epochs", type=int, default=100)
    p.add_argument("--model-name", default="wr-resnet", choices=sorted(MODEL_NAMES))
    p.add_argument("--load-raw", default=0, action="count",
                   help="train on the records' raw audio (GPU STFT / mel / mix_up) instead of their stored magnitude "
                        "spectrogram (audiomodel.py:2344-2349: count flag, default the spectrogram path)")
    p.add_argument("--multi-label", type=str2bool, default=False)
    p.add_argument("--n_mels", type=int, default=None)
    p.add_argument("--fmin", type=float, default=None)
    p.add_argument("--fmax", type=float, default=None)
    p.add_argument("--n_fft", type=int, default=None)
    p.add_argument("--break-freq", type=float, default=None)
    p.add_argument("-w", "--weights", help="model.pt, or a Keras *.weights.h5 / .keras file, to start from")
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--shuffle", type=str2bool, default=True)
    p.add_argument("--augment", type=str2bool, default=True, help="mix_up (tfdataset.py:473-481)")
    p.add_argument("--pcen", type=str2bool, default=True)
    # the reference trains in fp32 (MIXED_PRECISION = False, audiomodel.py:55-58);
    # bf16 is the mixed-precision policy it would otherwise set
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="fp32")
    p.add_argument("--steps-per-epoch", type=int, default=0)
    p.add_argument("--checkpoint-dir", default="checkpoints")
    p.add_argument("--seed", type=int, default=0)
    return p.parse_args(argv)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(process)d %(thread)s:%(levelname)7s %(message)s")
    train_model(parse_args())
