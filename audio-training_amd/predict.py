#!/usr/bin/env python3
"""Inference driver of the acfe path (reference predict.py:726-967,
predict_utils.py:9-239).

  python predict.py --file REC.wav CHECKPOINT_DIR [--stride 1] [--batch-size 1024]

The recording is decoded on the host (WAV via scipy; the reference's ffmpeg /
librosa loader and its track detection are out of scope), resampled to 48 kHz
and uploaded once; 3 s windows every `stride` seconds are read in place by the
fused front-end kernel (normalize, librosa-style centred STFT with constant
padding, |X|^2, mel; predict_utils.get_spect) and classified in batches.
The per-recording result is the mean of the window probabilities, thresholded
at 0.7 (predict.py:931-956).  Note: PCEN (if the model was trained with it)
normalises min/max over each window batch, as Keras predict does per batch.
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


class Predictor:
    def __init__(self, checkpoint_dir, device=None, dtype=None):
        from acfe.train import FrontEnd
        from audiomodel import build_model

        d = Path(checkpoint_dir)
        self.meta = json.loads((d / "metadata.txt").read_text())
        self.labels = self.meta["labels"]
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
    a = ap.parse_args(argv)
    p = Predictor(a.model)
    for f in a.file:
        t0 = time.perf_counter()
        r = p.predict_file(f, a.stride, a.batch_size, a.threshold)
        r["seconds"] = round(time.perf_counter() - t0, 3)
        print(json.dumps(r))


if __name__ == "__main__":
    main()
