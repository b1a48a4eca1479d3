"""custommel (reference custommel.py:1-61) for the acfe path.

`mel_f` is computed by the C restatement in libacfe (float64 math, float32
result; bit-exact with the reference on the golden vectors in tests/golden).
`mel_spec` applies it to a magnitude spectrogram on the host (used off the hot
path; the device path is acfe.frontend.MelPlan.mel)."""
from __future__ import annotations

import numpy as np

from acfe.frontend import mel_filterbank


def mel_f(sr, n_mels, fmin, fmax, n_fft, break_freq):
    """custommel.py:18-54: [n_mels, 1 + n_fft // 2] float32."""
    return mel_filterbank(sr, n_mels, fmin, fmax, n_fft, break_freq)


def mel_spec(stft, sr, n_fft, hop_length, n_mels, fmin, fmax, break_freq=1750, power=2):
    """custommel.py:57-61: mel_f(...) . |S|**power (float32 math, as the reference)."""
    magnitude = np.abs(stft) ** power
    return mel_f(sr, n_mels, fmin, fmax, n_fft, break_freq) @ magnitude
