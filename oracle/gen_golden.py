"""Generate golden mel-filterbank fixtures from the REFERENCE custommel.py.

Test infrastructure only (see oracle/__init__.py).  Run in the build container,
where /root/reference exists; the .npz outputs are committed under tests/golden/
and are the only thing that travels.  The reference imports `librosa` only for
`librosa.fft_frequencies` (custommel.py:24); librosa is absent here, so a stub
providing exactly that function (librosa's published definition:
`np.fft.rfftfreq(n_fft, 1/sr)`, i.e. linspace(0, sr/2, 1 + n_fft//2)) is injected.

Usage: python oracle/gen_golden.py [--ref /root/reference] [--out tests/golden]
"""
import argparse
import hashlib
import sys
import types
from pathlib import Path

import numpy as np


def _stub_librosa():
    mod = types.ModuleType("librosa")

    def fft_frequencies(*, sr=22050, n_fft=2048):
        return np.fft.rfftfreq(n=n_fft, d=1.0 / sr)

    mod.fft_frequencies = fft_frequencies
    sys.modules["librosa"] = mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parent.parent / "tests" / "golden"))
    a = ap.parse_args()
    _stub_librosa()
    sys.path.insert(0, a.ref)
    import custommel  # the reference module

    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    # configs used on the path: tfdataset.py:430-460 (fmin 100 / fmax 11000 /
    # n_fft 4096 / break 1000), module default tfdataset.py:46 (fmin 500),
    # n_fft<2048 -> 96 mels (tfdataset.py:448-452), predict default 160 mels.
    cfgs = [
        (48000, 128, 100, 11000, 4096, 1000),
        (48000, 160, 100, 11000, 4096, 1000),
        (48000, 160, 500, 11000, 4096, 1000),
        (48000, 96, 100, 11000, 1024, 1000),
        (48000, 64, 50, 8000, 2048, 1750),
    ]
    for sr, m, fmin, fmax, nfft, brk in cfgs:
        w = custommel.mel_f(sr, m, fmin, fmax, nfft, brk)
        rows, cols = np.nonzero(w)
        name = f"mel_f_sr{sr}_m{m}_f{fmin}-{fmax}_n{nfft}_b{brk}.npz"
        np.savez_compressed(
            out / name,
            params=np.array([sr, m, fmin, fmax, nfft, brk], dtype=np.float64),
            rows=rows.astype(np.int32),
            cols=cols.astype(np.int32),
            vals=w[rows, cols].astype(np.float32),
            shape=np.array(w.shape, dtype=np.int64),
            sha256=np.frombuffer(hashlib.sha256(np.ascontiguousarray(w).tobytes()).digest(), dtype=np.uint8),
        )
        print(name, w.shape, w.dtype, float(w.sum()), len(rows))
    # mel_spec on seeded synthetic |S| (power 1 and 2), custommel.py:57-61
    rng = np.random.default_rng(20260227)
    S = np.abs(rng.standard_normal((2049, 17)) + 1j * rng.standard_normal((2049, 17))).astype(np.float32)
    for p in (1, 2):
        y = custommel.mel_spec(S, 48000, 4096, 281, 128, 100, 11000, 1000, power=p)
        np.savez_compressed(out / f"mel_spec_p{p}.npz", S=S, mel=y)
        print("mel_spec", p, y.shape, y.dtype, float(y.sum()))


if __name__ == "__main__":
    main()
