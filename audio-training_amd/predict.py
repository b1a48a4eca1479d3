#!/usr/bin/env python3
"""Inference driver of the acfe path (reference predict.py:726-967,
predict_utils.py:9-239).

  python predict.py --file REC.wav CHECKPOINT_DIR [--stride 1] [--batch-size 1024]

The recording is decoded on the host (WAV via scipy; the reference's ffmpeg /
librosa loader is out of scope) and resampled to 48 kHz.

--mode tracks (default, the reference's predict.py:735-956): the digitally
silent tail is cut (get_end), signals are detected and merged into tracks on
the host (identifytracks.py), each track is cut into 3 s windows at a 1 s
stride (predict_utils.load_samples:59-150: short tracks centred in a 3 s
window, partial windows zero padded at a random offset), the windows of all
tracks go to the GPU as one batch (normalize, librosa-style centred STFT with
constant padding, |X|^2, mel, PCEN: predict_utils.get_spect) and the mean
sigmoid output per track is thresholded at 0.7, else the argmax becomes the
raw tag (predict.py:931-956).

--mode windows: the recording is uploaded once and 3 s windows every
`stride` seconds are read in place by the fused front-end kernel; the
per-recording result is the mean of the window probabilities.

Note: PCEN (if the model was trained with it) normalises min/max over each
window batch, as Keras predict does per batch.
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402

SR = 48000


def load_recording(path, sr=SR):
    """predict.load_recording (predict.py:59-66) for WAV input."""
    from scipy.io import wavfile
    from scipy.signal import resample_poly

    rate, data = wavfile.read(path)
    if np.issubdtype(data.dtype, np.integer):
        data = data.astype(np.float32) / float(np.iinfo(data.dtype).max)
    data = data.astype(np.float32)
    if data.ndim > 1:
        data = data.mean(1)
    if rate != sr:
        g = math.gcd(rate, sr)
        data = resample_poly(data, sr // g, rate // g).astype(np.float32)
    return data


class ModelResult:
    """predict.ModelResult (predict.py:1103-1120)."""

    def __init__(self, model):
        self.model = model
        self.labels, self.confidences = [], []
        self.raw_tag = self.raw_confidence = None

    def get_meta(self):
        meta = {"model": self.model, "species": self.labels, "likelihood": self.confidences}
        if self.raw_tag is not None:
            meta["raw_tag"] = self.raw_tag
            meta["raw_confidence"] = self.raw_confidence
        return meta


def track_windows(frames, sr, tracks, segment_length=3, stride=1, fmin=100, fmax=11000, pad_short_tracks=False,
                  rng=None):
    """The raw 3 s windows predict_utils.load_samples (:59-150) cuts from each
    track (before its normalize / spectrogram, which run on the GPU) ->
    list of [n_i, sr * segment_length] float32 arrays, one per track (empty
    for tracks wholly outside [fmin, fmax], which are not classified)."""
    rng = rng if rng is not None else np.random
    sample_size = int(sr * segment_length)
    frames = np.asarray(frames, np.float32)
    out = []
    for t in tracks:
        wins = []
        if t.freq_start is not None and t.freq_end is not None and (t.freq_start > fmax or t.freq_end < fmin):
            out.append(np.zeros((0, sample_size), np.float32))
            continue
        start, end = 0, segment_length
        sr_end, sr_start = int(t.end * sr), int(sr * t.start)
        if pad_short_tracks:
            end = min(end, t.length)  # predict_utils.py:75-77
            track_frames = frames[sr_start:sr_end]
        else:  # centre short tracks in one window
            missing = sample_size - (sr_end - sr_start)
            if missing > 0:
                offset = missing // 2
                sr_start -= offset
                if sr_start <= 0:
                    sr_start = 0
                    sr_end = min(sample_size, len(frames))
                else:
                    end_offset = sr_end + missing - offset
                    if end_offset > len(frames):
                        end_offset = len(frames)
                        sr_start = max(end_offset - sample_size, 0)
                    sr_end = end_offset
            track_frames = frames[sr_start:sr_end]
        sr_start, sr_end = 0, min(sr_end, sample_size)
        while True:
            data = track_frames[sr_start:sr_end]
            if len(data) != sample_size:
                extra = sample_size - len(data)
                off = int(rng.randint(0, extra))
                data = np.pad(data, (off, extra - off))
            wins.append(data)
            start += stride
            end = start + segment_length
            sr_start = int(start * sr)
            sr_end = min(int(end * sr), sr_start + sample_size)
            if end > t.length:  # always at least one window
                break
        out.append(np.stack(wins).astype(np.float32))
    return out


def detect_tracks(frames, sr=SR):
    """predict.main (:735-740): cut the silent tail, detect signals, merge
    them into tracks -> (tracks, frames[:end], end seconds)."""
    from identifytracks import get_end, get_tracks_from_signals, signal_noise

    end = get_end(frames, sr)
    frames = frames[: int(sr * end)]
    signals, _ = signal_noise(frames, sr)
    return get_tracks_from_signals(signals, end), frames, end


class Predictor:
    def __init__(self, checkpoint_dir, device=None, dtype=None):
        from acfe.train import FrontEnd
        from audiomodel import build_model

        d = Path(checkpoint_dir)
        self.meta = json.loads((d / "metadata.txt").read_text())
        self.labels = self.meta.get("ebird_labels") or self.meta["labels"]
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        dt = dtype or (torch.bfloat16 if self.meta.get("dtype", "bf16") == "bf16" else torch.float32)
        n_mels = self.meta.get("n_mels", 160)
        self.model = build_model(self.meta.get("name", "wr-resnet"), (n_mels, 513, 3), len(self.labels), dt)
        self.frontend = FrontEnd(n_mels=n_mels, n_fft=self.meta.get("n_fft", 4096), hop=self.meta.get("hop_length", 281),
                                 fmin=self.meta.get("fmin", 100), fmax=self.meta.get("fmax", 11000),
                                 break_freq=self.meta.get("break_freq", 1000), pcen=self.meta.get("pcen", True),
                                 dtype=dt, device=self.device, power=self.meta.get("power", 2))
        holder = torch.nn.ModuleList([self.frontend, self.model])
        if (d / "model.pt").exists():
            sd = torch.load(d / "model.pt", map_location="cpu", weights_only=True)
            holder.load_state_dict(sd)
        else:  # a reference checkpoint dir: {run}.keras / *.weights.h5 (predict.py:746-789)
            from keras_weights import load_keras_weights

            cands = sorted(d.glob("*.keras")) + sorted(d.glob("*.weights.h5"))
            if not cands:
                raise FileNotFoundError(f"{d}: no model.pt, *.keras or *.weights.h5")
            load_keras_weights(self.model, cands[0])
        holder.to(self.device).eval()

    @torch.no_grad()
    def predict_windows(self, recording: np.ndarray, stride=1.0, batch_size=1024, pad_mode="constant"):
        """Sigmoid outputs [n_windows, classes] for 3 s windows every `stride` s."""
        from acfe import ops

        n = SR * 3
        rec = np.asarray(recording, np.float32)
        if len(rec) < n:  # short recordings are zero padded to one window
            rec = np.pad(rec, (0, n - len(rec)))
        hop = int(round(stride * SR))
        n_win = 1 + (len(rec) - n) // hop
        dev_rec = torch.from_numpy(rec).to(self.device)
        out = []
        for first in range(0, n_win, batch_size):
            cnt = min(batch_size, n_win - first)
            feats = self.frontend.forward_windows(dev_rec, first, cnt, n=n, hop=hop, pad_mode=pad_mode)
            out.append(ops.sigmoid(self.model(feats)))
        return torch.cat(out).float().cpu().numpy()

    @torch.no_grad()
    def predict_clips(self, clips: np.ndarray, batch_size=1024):
        """Sigmoid outputs [B, classes] for raw [B, 144000] windows (each
        normalised on the GPU, centred STFT with constant padding)."""
        from acfe import ops

        out = []
        for a in range(0, len(clips), batch_size):
            x = torch.from_numpy(np.ascontiguousarray(clips[a:a + batch_size], np.float32)).to(self.device)
            out.append(ops.sigmoid(self.model(self.frontend(x, pad_mode="constant"))))
        return torch.cat(out).float().cpu().numpy()

    def predict_tracks(self, frames, threshold=None, batch_size=1024, rng=None):
        """Tracks of one recording with their ModelResult (predict.py:735-956)."""
        tracks, frames, end = detect_tracks(np.asarray(frames, np.float32))
        thresh = self.meta.get("threshold", 0.7) if threshold is None else threshold
        wins = track_windows(frames, SR, tracks, rng=rng)
        counts = [len(w) for w in wins]
        probs = self.predict_clips(np.concatenate(wins), batch_size) if sum(counts) else None
        at = 0
        for t, c in zip(tracks, counts):
            if c == 0:
                continue
            prediction = probs[at:at + c].mean(0)
            at += c
            r = ModelResult(self.meta.get("name", "wr-resnet"))
            t.predictions.append(r)
            max_p = None
            for i, p in enumerate(prediction):
                if max_p is None or p > max_p[1]:
                    max_p = (i, p)
                if p >= thresh:
                    r.labels.append(self.labels[i])
                    r.confidences.append(round(float(p) * 100))
            if not r.labels:
                r.raw_tag = self.labels[max_p[0]]
                r.raw_confidence = round(float(max_p[1]) * 100)
        return tracks, end

    def predict_file(self, path, stride=1.0, batch_size=1024, threshold=0.7):
        probs = self.predict_windows(load_recording(path), stride, batch_size)
        mean = probs.mean(0)
        labels = [(self.labels[i], float(mean[i])) for i in np.argsort(-mean) if mean[i] >= threshold]
        return {"file": str(path), "windows": int(probs.shape[0]), "labels": labels,
                "mean": {l: float(v) for l, v in zip(self.labels, mean)}}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("model", help="checkpoint dir (model.pt + metadata.txt from audiomodel.py)")
    ap.add_argument("--file", required=True, nargs="+")
    ap.add_argument("--stride", type=float, default=1.0)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--threshold", type=float, default=0.7)
    ap.add_argument("--mode", choices=("tracks", "windows"), default="tracks")
    a = ap.parse_args(argv)
    p = Predictor(a.model)
    for f in a.file:
        t0 = time.perf_counter()
        if a.mode == "tracks":
            tracks, end = p.predict_tracks(load_recording(f), a.threshold, a.batch_size)
            r = {"file": str(f), "end": end, "tracks": [t.get_meta() for t in tracks]}
        else:
            r = p.predict_file(f, a.stride, a.batch_size, a.threshold)
        r["seconds"] = round(time.perf_counter() - t0, 3)
        print(json.dumps(r, default=float))


if __name__ == "__main__":
    main()
