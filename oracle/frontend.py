"""Float64 numpy restatement of the reference feature front end (ORACLE, test-only).

Every function cites the reference file:line it restates.  See oracle/__init__.py
for who may import this module.
"""
from __future__ import annotations

import numpy as np

# ---------------------------------------------------------------- custommel.py


def hz_to_mel(frequencies, break_freq):
    """custommel.py:6-8 -- 2595*log10(1 + f/break_freq)."""
    frequencies = np.array(frequencies)
    return 2595.0 * np.log10(1.0 + frequencies / break_freq)


def mel_frequencies(n_mels, fmin, fmax, break_freq):
    """custommel.py:11-15."""
    lo = hz_to_mel(fmin, break_freq)
    hi = hz_to_mel(fmax, break_freq)
    mels = np.linspace(lo, hi, n_mels)
    return break_freq * (10.0 ** (mels / 2595.0) - 1.0)


def fft_frequencies(sr, n_fft):
    """librosa.fft_frequencies (used at custommel.py:24): rfftfreq(n_fft, 1/sr)."""
    return np.fft.rfftfreq(n=n_fft, d=1.0 / sr)


def mel_f(sr, n_mels, fmin, fmax, n_fft, break_freq):
    """custommel.py:18-54 -- [n_mels, 1 + n_fft//2] float32 triangular filterbank,
    Slaney area normalisation.  Reproduces the reference's float32 storage
    exactly: ramps are evaluated in float64, stored to float32, then scaled in
    place by the float64 `enorm` (numpy computes the in-place multiply in
    float64 and rounds once to float32)."""
    n_mels = int(n_mels)
    weights = np.zeros((n_mels, int(1 + n_fft // 2)), dtype=np.float32)
    fftfreqs = fft_frequencies(sr, n_fft)
    mf = mel_frequencies(n_mels + 2, fmin, fmax, break_freq)
    fdiff = np.diff(mf)
    ramps = np.subtract.outer(mf, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mf[2 : n_mels + 2] - mf[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def mel_spec(stft, sr, n_fft, hop_length, n_mels, fmin, fmax, break_freq=1750, power=2):
    """custommel.py:57-61 -- mel_f(...) . |S|**power."""
    magnitude = np.abs(stft) ** power
    return mel_f(sr, n_mels, fmin, fmax, n_fft, break_freq).dot(magnitude)


def mel_bands(weights):
    """Banded (CSR-like) view of a mel filterbank: per row (start, length, values).
    The reference applies the dense matrix (tfdataset.py:2049-2051); every row is a
    single contiguous run of non-zeros, so the banded product is the same sum."""
    starts, lens, vals = [], [], []
    for row in weights:
        nz = np.nonzero(row)[0]
        if len(nz) == 0:
            starts.append(0)
            lens.append(0)
            continue
        s, e = int(nz[0]), int(nz[-1]) + 1
        starts.append(s)
        lens.append(e - s)
        vals.append(row[s:e])
    return np.array(starts, np.int32), np.array(lens, np.int32), (np.concatenate(vals) if vals else np.zeros(0, np.float32))


# ---------------------------------------------------------------- tfdataset.py


def normalize(x):
    """tfdataset.py:1916-1934 (also predict_utils.py:153-160,
    audiodataset.py:1334-1341): per row x-min, /max, +1e-6, -0.5, *2."""
    x = np.asarray(x, dtype=np.float64)
    x = x - x.min(axis=-1, keepdims=True)
    with np.errstate(divide="ignore", invalid="ignore"):
        x = x / x.max(axis=-1, keepdims=True) + 0.000001
    return (x - 0.5) * 2


def normalize_f32(x):
    """The same in float32, operation for operation (predict_utils.py:153-160,
    audiodataset.py:1334-1341 -- numpy float32; tfdataset.py:1923-1929 has the
    same order in TF): pinned bit for bit to tests/golden/normalize_golden.npz,
    which oracle/gen_golden_normalize.py made with the reference functions."""
    x = np.asarray(x, dtype=np.float32)
    x = x - np.min(x, -1, keepdims=True)
    with np.errstate(divide="ignore", invalid="ignore"):
        x = x / np.max(x, -1, keepdims=True) + np.float32(0.000001)
    x = x - np.float32(0.5)
    return x * np.float32(2)


def mix_up_f32(x1, x2, lam):
    """tfdataset.py:950 image blend in float32 (x1 * l + x2 * (1 - l), one
    rounding per operation); lam [B]."""
    lam = np.asarray(lam, np.float32).reshape(-1, 1)
    return np.asarray(x1, np.float32) * lam + np.asarray(x2, np.float32) * (np.float32(1) - lam)


def mix_up(x1, y1, x2, y2, lam, single_label=True):
    """tfdataset.py:930-955 with the per-row lambda supplied (the reference draws
    it from Beta(a,a)*Bernoulli(chance), :942-946)."""
    lam = np.asarray(lam, dtype=np.float64).reshape(-1, 1)
    x = np.asarray(x1, np.float64) * lam + np.asarray(x2, np.float64) * (1 - lam)
    yl = (lam > 0.5).astype(np.float64) if single_label else lam
    y = np.asarray(y1, np.float64) * yl + np.asarray(y2, np.float64) * (1 - yl)
    return x, y


def hann_periodic(n):
    """tf.signal.hann_window(n, periodic=True) == scipy hann(n, sym=False)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def num_frames_pad_end(n, hop):
    """tf.signal.frame(pad_end=True): ceil(n / hop) frames."""
    return -(-n // hop)


def stft_pad_end(x, n_fft=4096, hop=281):
    """tf.signal.stft(x, n_fft, hop, fft_length=n_fft, hann_window, pad_end=True)
    (tfdataset.py:2026-2034): [B, T, 1+n_fft//2] complex128."""
    x = np.atleast_2d(np.asarray(x, np.float64))
    b, n = x.shape
    t = num_frames_pad_end(n, hop)
    total = (t - 1) * hop + n_fft
    xp = np.zeros((b, max(total, n)), np.float64)
    xp[:, :n] = x
    idx = np.arange(t)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = xp[:, idx] * hann_periodic(n_fft)
    return np.fft.rfft(frames, axis=-1)


def stft_center(x, n_fft=4096, hop=281, pad_mode="constant"):
    """librosa.stft(x, n_fft, hop, center=True) as used at predict_utils.py:194
    (librosa >= 0.10 default pad_mode 'constant'; 'reflect' before 0.10):
    [B, 1+n_fft//2, T] complex128 with T = 1 + n//hop."""
    x = np.atleast_2d(np.asarray(x, np.float64))
    b, n = x.shape
    pad = n_fft // 2
    xp = np.pad(x, ((0, 0), (pad, pad)), mode=pad_mode)
    t = 1 + (xp.shape[1] - n_fft) // hop
    idx = np.arange(t)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = xp[:, idx] * hann_periodic(n_fft)
    return np.transpose(np.fft.rfft(frames, axis=-1), (0, 2, 1))


def raw_to_mel(raw, weights, n_fft=4096, hop=281, power=2):
    """tfdataset.py:2007-2059 without the final repeat: |stft|^power -> mel.
    Returns [B, M, T] float64 (the reference returns [B, M, T, 3] of identical
    channels, tfdataset.py:2052-2053)."""
    s = np.abs(stft_pad_end(raw, n_fft, hop)) ** power  # [B,T,F]
    return np.einsum("mf,btf->bmt", weights.astype(np.float64), s)


def get_spect(data, weights, n_fft=4096, hop=281, power=2, pad_mode="constant"):
    """predict_utils.py:163-239 (htk branch): mel_spec(|librosa.stft(center)|, power)."""
    s = np.abs(stft_center(data, n_fft, hop, pad_mode)) ** power  # [B,F,T]
    return np.einsum("mf,bft->bmt", weights.astype(np.float64), s)


# ---------------------------------------------------------------- tfpcen.py

PCEN_DEFAULTS = dict(gain=0.98, bias=2.0, root=2.0, smooth=0.04, eps=1e-6)


def ema(x_btm, w):
    """tfpcen.py:33-39: tf.scan over axis 1 with initializer x[:,0]:
    a_t = w x_t + (1-w) a_{t-1}, a_{-1} = x_0.  Input [B,T,M]."""
    w = float(np.clip(w, 0.0, 1.0))
    x = np.asarray(x_btm, np.float64)
    out = np.empty_like(x)
    a = x[:, 0]
    for t in range(x.shape[1]):
        a = w * x[:, t] + (1.0 - w) * a
        out[:, t] = a
    return out


def pcen_unnormalised(x_btm, gain=0.98, bias=2.0, root=2.0, smooth=0.04, eps=1e-6):
    """tfpcen.py:89-95 before normalize_minmax."""
    g = min(gain, 1.0)
    r = max(root, 1.0)
    m = ema(x_btm, smooth)
    x = np.asarray(x_btm, np.float64)
    return (x / (eps + m) ** g + bias) ** (1.0 / r) - bias ** (1.0 / r)


def normalize_minmax(d):
    """tfpcen.py:105-110: global (whole tensor) min/max to [-1, 1]."""
    d = np.asarray(d, np.float64)
    mx, mn = d.max(), d.min()
    return 2 * ((d - mn) / (mx - mn)) - 1


def pcen(x_btm, **p):
    """tfpcen.py:89-99 (PCEN.call) on [B,T,M]."""
    return normalize_minmax(pcen_unnormalised(x_btm, **p))
