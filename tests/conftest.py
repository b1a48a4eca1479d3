import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "audio-training_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def synth_clips(b, n=144000, sr=48000, seed=20260227, noise_only_every=0):
    """SURVEY.md 8(d) synthetic clips: 1-3 linear chirps + white noise, clipped to [-1, 1]."""
    import numpy as np

    out = np.zeros((b, n), np.float32)
    t = np.arange(n) / sr
    for i in range(b):
        rng = np.random.default_rng(seed + i)
        x = rng.normal(0, rng.uniform(0.002, 0.02), n)
        if not (noise_only_every and i % noise_only_every == 0):
            for _ in range(rng.integers(1, 4)):
                f0, f1 = rng.uniform(500, 10000, 2)
                amp = rng.uniform(0.05, 0.5)
                on = rng.uniform(0, 2.0)
                dur = rng.uniform(0.3, 3.0 - on)
                m = (t >= on) & (t < on + dur)
                tt = t[m] - on
                x[m] += amp * np.sin(2 * np.pi * (f0 * tt + 0.5 * (f1 - f0) / dur * tt * tt))
        out[i] = np.clip(x, -1, 1)
    return out
