"""Input pipeline of the acfe path (reference tfdataset.py:193-506, :983-1228).

get_dataset(dir, labels, global_epoch=None, **args) keeps the reference
signature and return tuple (dataset, remapped, epoch_size, labels,
extra_label_map).  The dataset reads the GZIP TFRecord shards of `dir`
(audio/raw [144000] f32, audio/class/text, ...; tfdataset.py:1005-1060) with a
pool of reader threads (zlib releases the GIL), assembles batches in pinned
host memory and hands out DEVICE tensors: x [B, 144000] fp32 raw audio (the
normalize / mix_up / STFT / mel work happens on the GPU, acfe.train.FrontEnd)
and y [B, len(labels)] one-hot.  With augment=True each item is a pair of
batches for mix_up (tfdataset.py:473-481).
"""
from __future__ import annotations

import logging
import queue
import random
import threading
from pathlib import Path

import numpy as np
import torch

import tfrecord as tfr

N_SAMPLES = 48000 * 3
HOP_LENGTH, NFFT, SR, BREAK_FREQ, FMIN, FMAX = 281, 4096, 48000, 1000, 100, 11000  # tfdataset.py:42-56
N_MELS = 160
DIMENSIONS = (160, 513, 1)


class AudioDataset:
    """Iterable over device batches; one pass = one epoch."""

    def __init__(self, files, labels, batch_size=32, shuffle=True, augment=False, device=None, threads=8,
                 drop_remainder=False, seed=0, label_map=None, record_shard=None, load_raw=True):
        """record_shard=(rank, world): keep only the records whose (file index
        + record index) % world == rank -- data-parallel sharding when there
        are fewer shard files than ranks (otherwise ranks take whole files).
        load_raw=False: batches of the stored magnitude spectrograms
        [B, 2049, 513] (audio/spectogram, tfdataset.py:1032-1034, 1081-1082);
        there is no mix_up on that path (tfdataset.py:503-504)."""
        self.files, self.labels = list(files), list(labels)
        self.record_shard = record_shard
        self.load_raw = load_raw
        if not load_raw:
            augment = False
        self.batch_size, self.shuffle, self.augment = batch_size, shuffle, augment
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.threads, self.drop_remainder, self.seed = threads, drop_remainder, seed
        self.label_index = {l: i for i, l in enumerate(self.labels)}
        self.label_map = label_map or {}
        self.epoch = 0

    def _examples(self, files):
        q: queue.Queue = queue.Queue(maxsize=4 * self.batch_size)
        DONE = object()
        idx = iter(range(len(files)))
        lock = threading.Lock()
        stable = {f: i for i, f in enumerate(self.files)}
        shard = self.record_shard

        def worker():
            while True:
                with lock:
                    i = next(idx, None)
                if i is None:
                    q.put(DONE)
                    return
                for r, rec in enumerate(tfr.read_records(files[i], ignore_errors=True)):  # tfdataset.py:226
                    if shard is not None and (stable.get(files[i], i) + r) % shard[1] != shard[0]:
                        continue
                    ex = tfr.parse_audio_example(rec, load_raw=self.load_raw)
                    x = ex["raw"] if self.load_raw else ex["spectrogram"]
                    if not np.all(np.isfinite(x)):  # NaN/Inf filter, tfdataset.py:297
                        continue
                    lab = self.label_map.get(ex["text"], ex["text"])
                    if lab not in self.label_index:
                        continue
                    q.put((x, self.label_index[lab]))

        ts = [threading.Thread(target=worker, daemon=True) for _ in range(min(self.threads, max(1, len(files))))]
        for t in ts:
            t.start()
        live = len(ts)
        while live:
            item = q.get()
            if item is DONE:
                live -= 1
                continue
            yield item

    def _batches(self):
        files = list(self.files)
        rng = random.Random(self.seed + self.epoch)
        if self.shuffle:
            rng.shuffle(files)
        buf = []
        pool = []
        for ex in self._examples(files):
            pool.append(ex)
            if self.shuffle and len(pool) < 4 * self.batch_size:  # shuffle buffer, tfdataset.py:835-890
                continue
            j = rng.randrange(len(pool)) if self.shuffle else 0
            buf.append(pool.pop(j))
            if len(buf) == self.batch_size:
                yield buf
                buf = []
        while pool:
            buf.append(pool.pop(rng.randrange(len(pool)) if self.shuffle else 0))
            if len(buf) == self.batch_size:
                yield buf
                buf = []
        if buf and not self.drop_remainder:
            yield buf

    def _to_device(self, items):
        b = len(items)
        pin = torch.device(self.device).type == "cuda"
        x = torch.empty((b,) + tuple(items[0][0].shape), dtype=torch.float32, pin_memory=pin)
        y = torch.zeros((b, len(self.labels)), dtype=torch.float32, pin_memory=pin)
        for i, (raw, lab) in enumerate(items):
            x[i] = torch.from_numpy(raw)
            y[i, lab] = 1.0
        return x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)

    def __iter__(self):
        it = self._batches()
        self.epoch += 1
        if not self.augment:
            for items in it:
                yield self._to_device(items)
            return
        # second independent pass over the data for mix_up (tfdataset.py:473-480)
        other = AudioDataset(self.files, self.labels, self.batch_size, True, False, self.device, self.threads,
                             self.drop_remainder, self.seed + 7919 * self.epoch, self.label_map, self.record_shard,
                             self.load_raw)
        for a, b in zip(it, other._batches()):
            if len(a) != len(b):
                break
            yield self._to_device(a), self._to_device(b)

    def __len__(self):
        return -1


def _files(dir):
    d = Path(dir)
    files = sorted(d.glob("*.tfrecord")) or sorted(d.rglob("*.tfrecord"))
    return [str(f) for f in files]


def count_examples(dir) -> int:
    return sum(1 for f in _files(dir) for _ in tfr.read_records(f, ignore_errors=True))


def get_dataset(dir, labels, global_epoch=None, **args):
    """tfdataset.get_dataset (tfdataset.py:429-506) -> (dataset, remapped, epoch_size, labels, extra_label_map)."""
    global N_MELS, FMIN, FMAX, NFFT, BREAK_FREQ
    if args.get("n_mels"):
        N_MELS = args["n_mels"]
    if args.get("fmin") is not None:
        FMIN, FMAX = args.get("fmin", FMIN), args.get("fmax", FMAX)
    if args.get("n_fft") is not None:
        NFFT = args["n_fft"]
    if args.get("break_freq") is not None:
        BREAK_FREQ = args["break_freq"]
    files = _files(dir)
    if not files:
        raise FileNotFoundError(f"no *.tfrecord under {dir}")
    labels = list(labels)
    remapped = {l: [l] for l in labels}
    epoch_size = args.get("epoch_size") or None
    ds = AudioDataset(files, labels, batch_size=args.get("batch_size", 32), shuffle=args.get("shuffle", True),
                      augment=args.get("augment", False), device=args.get("device"),
                      threads=args.get("threads", 8), seed=args.get("seed", 0),
                      label_map=args.get("label_map"), load_raw=args.get("load_raw", True))
    logging.info("dataset %s: %d shards, %d labels", dir, len(files), len(labels))
    return ds, remapped, epoch_size, labels, {}
