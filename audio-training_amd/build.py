#!/usr/bin/env python3
"""Dataset builder of the acfe path (reference build.py:679-814, audiowriter.py).

Writes GZIP TFRecord shards of 3 s @ 48 kHz samples in the reference schema
(audiowriter.create_tf_example, audiowriter.py:67-174) into
<out>/training-data/{train,validation,test}/ and the training-meta.json that
audiomodel.py reads (build.py:795-814: labels, type, counts{split:{rec_counts,
sample_counts}}, recs, ... plus the feature config).

Sources (the reference's recording curation, track detection and eBird
taxonomy are out of scope):
  --synthetic N --labels bird,noise   SURVEY.md 8(d) chirp+noise clips ("noise" = noise only)
  -d DIR                              DIR/<label>/*.wav, resampled to 48 kHz, cut into
                                      3 s samples every --stride seconds
Splits are made per recording (no recording in two splits, build.py:817-837).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
from collections import Counter, defaultdict
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import tfrecord as tfr  # noqa: E402

SR = 48000
SEGMENT = 3


def synth_clip(rng, noise_only, n=SR * SEGMENT):
    t = np.arange(n) / SR
    x = rng.normal(0, rng.uniform(0.002, 0.02), n)
    if not noise_only:
        for _ in range(rng.integers(1, 4)):
            f0, f1 = rng.uniform(500, 10000, 2)
            amp, on = rng.uniform(0.05, 0.5), rng.uniform(0, 2.0)
            dur = rng.uniform(0.3, SEGMENT - on)
            m = (t >= on) & (t < on + dur)
            tt = t[m] - on
            x[m] += amp * np.sin(2 * np.pi * (f0 * tt + 0.5 * (f1 - f0) / dur * tt * tt))
    return np.clip(x, -1, 1).astype(np.float32)


def synthetic_samples(n, labels, seed=20260227, clips_per_rec=4):
    """(rec_id, label, start_s, raw) tuples; `clips_per_rec` samples share a recording id."""
    out = []
    for i in range(n):
        rng = np.random.default_rng(seed + i)
        lab = labels[i % len(labels)]
        out.append((f"syn{i // clips_per_rec:06d}_{lab}", lab, float(i % clips_per_rec), synth_clip(rng, lab == "noise")))
    return out


def wav_samples(root, stride=1.0):
    from scipy.io import wavfile
    from scipy.signal import resample_poly

    out = []
    for wav in sorted(Path(root).rglob("*.wav")):
        lab = wav.parent.name
        sr, data = wavfile.read(wav)
        data = data.astype(np.float32)
        if data.ndim > 1:
            data = data.mean(1)
        if np.issubdtype(data.dtype, np.integer) or np.abs(data).max() > 1.5:
            data = data / max(1.0, float(np.abs(data).max()))
        if sr != SR:
            g = math.gcd(sr, SR)
            data = resample_poly(data, SR // g, sr // g).astype(np.float32)
        n = SR * SEGMENT
        if len(data) < n:  # random-offset pad as predict_utils.load_samples (:116-119)
            off = (n - len(data)) // 2
            data = np.pad(data, (off, n - len(data) - off))
        start = 0
        while start + n <= len(data):
            out.append((wav.stem, lab, start / SR, data[start:start + n]))
            start += int(stride * SR)
    return out


def split_by_recording(samples, fractions=(0.8, 0.1, 0.1), seed=0):
    recs = sorted({s[0] for s in samples})
    rng = np.random.default_rng(seed)
    rng.shuffle(recs)
    n = len(recs)
    n_tr = max(1, int(round(fractions[0] * n)))
    n_va = max(1 if n > 2 else 0, int(round(fractions[1] * n)))
    parts = {"train": set(recs[:n_tr]), "validation": set(recs[n_tr:n_tr + n_va]), "test": set(recs[n_tr + n_va:])}
    return {k: [s for s in samples if s[0] in v] for k, v in parts.items()}


def normalize_data(x):
    """audiodataset.normalize_data (audiodataset.py:1334-1341)."""
    x = x - np.min(x, -1, keepdims=True)
    x = x / np.max(x, -1, keepdims=True) + 0.000001
    return (x - 0.5) * 2


def stft_magnitude(clip, n_fft=4096, hop=281):
    """The stored spectrogram of audiodataset.load_data (:1302-1303):
    |librosa.stft(normalize_data(clip), n_fft, hop)| with librosa's defaults
    (center=True, constant padding as of librosa 0.10, periodic Hann window)
    -> float32 [1 + n_fft // 2, 1 + len // hop]."""
    x = normalize_data(np.asarray(clip, np.float64))
    x = np.pad(x, (n_fft // 2, n_fft // 2))
    t = 1 + (len(x) - n_fft) // hop
    win = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n_fft) / n_fft)
    out = np.empty((n_fft // 2 + 1, t), np.float32)
    for a in range(0, t, 64):  # bounded frame blocks (64 x 4096 doubles)
        idx = np.arange(a, min(t, a + 64))[:, None] * hop + np.arange(n_fft)[None, :]
        out[:, a:a + idx.shape[0]] = np.abs(np.fft.rfft(x[idx] * win, axis=-1)).T
    return out


def write_split(samples, out_dir, shards=4, spectrogram=True):
    out_dir.mkdir(parents=True, exist_ok=True)
    writers = [tfr.TFRecordWriter(out_dir / f"{i:05d}.tfrecord") for i in range(max(1, shards))]
    for i, (rec, lab, start, raw) in enumerate(samples):
        spec = stft_magnitude(raw) if spectrogram else None
        writers[i % len(writers)].write(tfr.audio_example(raw, rec, i, lab, lab, start_s=start, spectrogram=spec))
    for w in writers:
        w.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("out", help="output base dir (records go to <out>/training-data)")
    ap.add_argument("-d", "--dir", help="directory of <label>/*.wav recordings")
    ap.add_argument("--synthetic", type=int, default=0, help="number of synthetic 3 s clips")
    ap.add_argument("--labels", default="bird,noise")
    ap.add_argument("--stride", type=float, default=1.0, help="segment stride (s)")
    ap.add_argument("-m", "--mels", type=int, default=160)
    ap.add_argument("-b", "--break-freq", type=float, default=1000)
    ap.add_argument("--hop-length", type=int, default=281)
    ap.add_argument("--fmin", type=float, default=100)
    ap.add_argument("--fmax", type=float, default=11000)
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-spectrogram", action="store_true",
                    help="store audio/raw only (the reference also stores audio/spectogram, audiowriter.py:131-134, "
                         "which the default load_raw=False training path reads)")
    a = ap.parse_args(argv)
    if a.synthetic:
        samples = synthetic_samples(a.synthetic, a.labels.split(","), seed=20260227 + a.seed)
    elif a.dir:
        samples = wav_samples(a.dir, a.stride)
    else:
        ap.error("need --synthetic N or -d DIR")
    labels = sorted({s[1] for s in samples})
    splits = split_by_recording(samples, seed=a.seed)
    for x in ("validation", "test"):  # validate_datasets (build.py:817-837)
        assert not ({s[0] for s in splits["train"]} & {s[0] for s in splits[x]})
    base = Path(a.out) / "training-data"
    counts, recs = {}, {}
    for name, ss in splits.items():
        write_split(ss, base / name, a.shards, spectrogram=not a.no_spectrogram)
        rc = defaultdict(set)
        for s in ss:
            rc[s[1]].add(s[0])
        counts[name] = {"rec_counts": {k: len(v) for k, v in rc.items()},
                        "sample_counts": dict(Counter(s[1] for s in ss))}
        recs[name] = sorted({s[0] for s in ss})
    meta = {"labels": labels, "type": "audio", "counts": counts, "recs": recs, "by_label": False, "relabbled": False,
            "segment_length": SEGMENT, "segment_stride": a.stride, "hop_length": a.hop_length, "n_mels": a.mels,
            "fmin": a.fmin, "fmax": a.fmax, "break_freq": a.break_freq, "sample_rate": SR, "n_fft": 4096}
    with open(base / "training-meta.json", "w") as f:
        json.dump(meta, f, indent=4)
    print(json.dumps({k: v["sample_counts"] for k, v in counts.items()}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
