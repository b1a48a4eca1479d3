"""Generate golden fixtures for the clip normalisation
from the REFERENCE itself.

Test infrastructure only (see oracle/__init__.py).  Run in the build container,
where /root/reference exists; only the .npz output (tests/golden/) travels.

The reference normalises a clip in three places with the same float32
operation order -- subtract the min, divide by the (new) max, + 1e-6, - 0.5,
* 2:

  * tfdataset.normalize (tfdataset.py:1916-1934, TF ops; TF is absent here),
  * predict_utils.normalize_data (predict_utils.py:153-160, numpy float32),
  * audiodataset.normalize_data (audiodataset.py:1334-1341, numpy float32).

The two numpy ones are importable with empty stub modules for the heavy
imports their modules never use in these functions (librosa gets
`fft_frequencies` for custommel, as in oracle/gen_golden.py).  Pinned:

  * both normalize_data functions on seeded float32 clips (three 3 s @ 48 kHz
    clips of int16-quantised hash noise + a chirp at different gains, a
    constant clip -- 0 / 0 gives NaN --, a 5 000-sample clip and a lone spike);
    both reference functions must agree bit for bit;
  * predict_utils.load_samples(normalize=True) (:9-150) on a 20 s recording
    with the window cutting of tests/golden/tracks_golden.npz case 0 / 1: the
    zero-padded short windows are normalised after padding, so the pad zeros
    take part in the min / max.

Outputs of 144 000-sample clips are stored as the SHA-256 of their float32
bytes (bit-exact pin) plus every 97th value (for diagnostics); short clips in
full.  Inputs are rebuilt by the test from `hash_audio` below (integer
arithmetic, identical on every machine).

Usage: python oracle/gen_golden_normalize.py [--ref /root/reference] [--out tests/golden]
"""
import argparse
import hashlib
import sys
import types
from pathlib import Path

import numpy as np

SR = 48000
N = 3 * SR
STRIDE = 97


def hash_audio(n, seed, gain):
    """float32 clip: int16 hash noise (splitmix-style, exact uint64 math) at a
    quarter scale plus a quantised chirp, times a float32 gain."""
    i = np.arange(n, dtype=np.uint64) + (np.full(1, seed, np.uint64) * np.uint64(0x9E3779B97F4A7C15))[0]
    z = (i ^ (i >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    noise = (z >> np.uint64(48)).astype(np.int64) - 32768  # [-32768, 32767]
    t = np.arange(n, dtype=np.int64)
    # integer-phase chirp, quantised to int16 (numpy's sin of the same f64
    # argument is what both sides compute; the test only needs it reproducible
    # on one machine -- the fixture stores the outputs, the test the recipe)
    chirp = np.round(12000.0 * np.sin(2 * np.pi * (500.0 + 0.01 * t) * t / SR)).astype(np.int64)
    q = np.clip(noise // 4 + chirp, -32768, 32767).astype(np.float32) / np.float32(32768.0)
    return (q * np.float32(gain)).astype(np.float32)


def clip_set():
    """name -> float32 1-D clip (the test rebuilds the same set)."""
    spike = np.zeros(N, np.float32)
    spike[12345] = np.float32(0.75)
    return {
        "full0": hash_audio(N, 1, 1.0),
        "full1": hash_audio(N, 2, 0.037),
        "full2": hash_audio(N, 3, 3.5),
        "const": np.full(2000, 0.25, np.float32),
        "short": hash_audio(5000, 4, 0.5),
        "spike": spike,
    }


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def _stubs():
    lib = types.ModuleType("librosa")
    lib.fft_frequencies = lambda *, sr=22050, n_fft=2048: np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    lib.display = types.ModuleType("librosa.display")
    sys.modules["librosa"] = lib
    sys.modules["librosa.display"] = lib.display
    for name in ("cv2", "plot_utils", "tensorflow", "soundfile", "matplotlib", "matplotlib.pyplot", "audioread",
                 "audioread.ffdec"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["matplotlib"].pyplot = sys.modules["matplotlib.pyplot"]
    sys.modules["audioread"].ffdec = sys.modules["audioread.ffdec"]
    ut = types.ModuleType("utils")  # the reference's utils.py (eBird maps): not on this path
    for f in ("get_label_to_ebird_map", "get_ebird_id", "get_ebird_ids_to_labels"):
        setattr(ut, f, lambda *a, **k: None)
    sys.modules["utils"] = ut


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parent.parent / "tests" / "golden"))
    a = ap.parse_args()
    _stubs()
    sys.path.insert(0, a.ref)
    import audiodataset as ad
    import identifytracks as it
    import predict_utils as pu

    out = {}
    clips = clip_set()
    with np.errstate(divide="ignore", invalid="ignore"):
        for name, x in clips.items():
            y = pu.normalize_data(x)
            y2 = ad.normalize_data(x)
            assert y.dtype == np.float32 and y2.dtype == np.float32
            assert y.tobytes() == y2.tobytes(), name  # the two reference copies agree bit for bit
            if len(x) == N:
                out[f"norm_{name}_sha"] = np.array(sha(y))
                out[f"norm_{name}_sample"] = y[::STRIDE].copy()
            else:
                out[f"norm_{name}"] = y
        # a [3, N] batch normalised along the last axis (the batched call
        # tfdataset.normalize makes) == the three clips one by one
        batch = np.stack([clips["full0"], clips["full1"], clips["full2"]])
        yb = pu.normalize_data(batch)
        for r, name in enumerate(("full0", "full1", "full2")):
            assert sha(yb[r]) == str(out[f"norm_{name}_sha"]), name

    # load_samples(normalize=True): the window layout from a ramp run (as
    # gen_golden_tracks.py), the normalised windows from a hash-noise run with
    # the same np.random seed (same pad offsets)
    pu.get_spect = lambda data, *args, **kw: np.array(data, copy=True)
    rows, hashes, samples = [], [], []
    for k, (secs, boxes, pad, seed) in enumerate([
        (20, [(5.0, 6.2), (2.0, 7.5), (0.2, 1.0), (19.3, 19.9), (18.0, 20.0), (0.0, 3.0), (4.0, 4.05)], False, 10),
        (20, [(5.0, 6.2), (2.0, 7.5), (0.2, 1.0), (19.3, 19.9), (18.0, 20.0), (0.0, 3.0), (4.0, 4.05)], True, 11),
    ]):
        n = SR * secs
        tracks = [it.Signal(s, e, 1000.0, 3000.0, 1) for s, e in boxes]
        np.random.seed(seed)
        lay = pu.load_samples(np.arange(1, n + 1, dtype=np.float32), SR, tracks, normalize=False,
                              pad_short_tracks=pad)
        rec = hash_audio(n, 100 + k, 0.8)
        np.random.seed(seed)
        res = pu.load_samples(rec, SR, tracks, normalize=True, pad_short_tracks=pad)
        for ti, (wl, wn) in enumerate(zip(lay, res)):
            assert len(wl) == len(wn)
            for w, y in zip(wl, wn):
                w, y = np.asarray(w), np.asarray(y, np.float32)
                nz = np.flatnonzero(w)
                first, cnt = int(nz[0]), len(nz)
                src = int(w[first]) - 1
                win = np.zeros(N, np.float32)
                win[first:first + cnt] = rec[src:src + cnt]
                assert pu.normalize_data(win).tobytes() == y.tobytes()
                rows.append((k, ti, first, src, cnt))
                hashes.append(sha(y))
                samples.append(y[::STRIDE])
    out.update(ls_rows=np.array(rows, np.int64), ls_sha=np.array(hashes), ls_sample=np.stack(samples))
    print("normalize clips", len(clips), "load_samples windows", len(rows))
    dst = Path(a.out) / "normalize_golden.npz"
    np.savez_compressed(dst, **out)
    print("wrote", dst)


if __name__ == "__main__":
    main()
