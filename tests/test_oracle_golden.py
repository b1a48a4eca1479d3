"""Pin the CPU oracle (and the C restatement of mel_f) against golden vectors
generated from the reference custommel.py itself (oracle/gen_golden.py)."""
import hashlib

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import frontend as of

MEL_FILES = sorted(GOLDEN.glob("mel_f_*.npz"))


def _dense(z):
    w = np.zeros(tuple(z["shape"]), np.float32)
    w[z["rows"], z["cols"]] = z["vals"]
    return w


@pytest.mark.parametrize("path", MEL_FILES, ids=lambda p: p.stem)
def test_oracle_mel_f_bitexact(path):
    z = np.load(path)
    sr, m, fmin, fmax, nfft, brk = z["params"]
    w = of.mel_f(int(sr), int(m), fmin, fmax, int(nfft), brk)
    ref = _dense(z)
    assert w.dtype == np.float32 and w.shape == ref.shape
    assert np.array_equal(w, ref)
    assert hashlib.sha256(np.ascontiguousarray(w).tobytes()).digest() == bytes(z["sha256"])


@pytest.mark.parametrize("path", MEL_FILES, ids=lambda p: p.stem)
def test_c_mel_filterbank_bitexact(path):
    """libacfe's acfe_mel_filterbank (host C, no GPU needed) vs the reference."""
    from acfe.frontend import mel_filterbank

    z = np.load(path)
    sr, m, fmin, fmax, nfft, brk = z["params"]
    w = mel_filterbank(int(sr), int(m), fmin, fmax, int(nfft), brk)
    assert np.array_equal(w, _dense(z))


def test_golden_band_structure():
    z = np.load(GOLDEN / "mel_f_sr48000_m128_f100-11000_n4096_b1000.npz")
    w = _dense(z)
    st, ln, vals = of.mel_bands(w)
    assert len(z["vals"]) == 1839
    assert st.min() == 9 and (st + ln).max() - 1 == 938
    assert ln.max() <= 37
    # every row is one contiguous run: banded product == dense product
    s = np.random.default_rng(0).random((2049, 5))
    dense = w.astype(np.float64) @ s
    band = np.stack([vals[ln[:i].sum(): ln[: i + 1].sum()].astype(np.float64) @ s[st[i]: st[i] + ln[i]]
                     for i in range(len(st))])
    np.testing.assert_allclose(band, dense, rtol=1e-12, atol=0)


@pytest.mark.parametrize("p", [1, 2])
def test_oracle_mel_spec(p):
    z = np.load(GOLDEN / f"mel_spec_p{p}.npz")
    y = of.mel_spec(z["S"], 48000, 4096, 281, 128, 100, 11000, 1000, power=p)
    np.testing.assert_allclose(y, z["mel"], rtol=2e-6, atol=1e-6 * np.abs(z["mel"]).max())


def test_stft_pad_end_matches_direct_dft():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 3000))
    n_fft, hop = 256, 97
    X = of.stft_pad_end(x, n_fft, hop)
    t = of.num_frames_pad_end(3000, hop)
    assert X.shape == (2, t, 129) and t == -(-3000 // hop)
    win = of.hann_periodic(n_fft)
    for f in (0, t // 2, t - 1):
        seg = np.zeros(n_fft)
        s = x[1, f * hop: f * hop + n_fft]
        seg[: len(s)] = s
        k = np.arange(129)[:, None] * np.arange(n_fft)[None, :]
        d = (np.exp(-2j * np.pi * k / n_fft) * (seg * win)[None, :]).sum(1)
        np.testing.assert_allclose(X[1, f], d, rtol=1e-9, atol=1e-9)


def test_stft_shapes_reference_config():
    # tfdataset.py:2026: 144000 samples, n_fft 4096, hop 281 -> 513 frames, 3968 zeros padded
    assert of.num_frames_pad_end(144000, 281) == 513
    assert (513 - 1) * 281 + 4096 - 144000 == 3968
    X = of.stft_center(np.zeros((1, 144000)), 4096, 281)
    assert X.shape == (1, 2049, 513)


def test_normalize_range():
    x = np.random.default_rng(2).standard_normal((3, 1000))
    y = of.normalize(x)
    assert np.allclose(y.min(1), 2 * (1e-6 - 0.5))
    assert np.allclose(y.max(1), 2 * (1 + 1e-6 - 0.5))


def test_pcen_oracle_consistency():
    """numpy and torch-f64 PCEN restatements agree; output spans [-1, 1]."""
    import torch

    from oracle.torch_ref import pcen_torch

    x = np.random.default_rng(3).random((2, 40, 8)) * 10
    ref = of.pcen(x)
    out = pcen_torch(torch.from_numpy(x), torch.tensor([0.98, 2.0, 2.0, 0.04], dtype=torch.float64))
    np.testing.assert_allclose(out.numpy(), ref.transpose(0, 2, 1), rtol=1e-12, atol=1e-12)
    assert ref.min() == -1 and ref.max() == 1


def test_ema_initializer_semantics():
    # tf.scan(initializer=x[:,0]) -> first output equals x_0 exactly
    x = np.random.default_rng(4).random((1, 5, 2))
    e = of.ema(x, 0.3)
    np.testing.assert_allclose(e[:, 0], x[:, 0])
    np.testing.assert_allclose(e[:, 1], 0.3 * x[:, 1] + 0.7 * x[:, 0])


# ---------------------------------------------------------------- normalize
def _norm_golden():
    return np.load(GOLDEN / "normalize_golden.npz")


def test_oracle_normalize_f32_bitexact():
    """of.normalize_f32 against the reference predict_utils / audiodataset
    normalize_data outputs (oracle/gen_golden_normalize.py): every clip of the
    set bit for bit (SHA-256 of the float32 bytes for the 3 s clips, the
    values themselves for the short ones; the constant clip is 0 / 0 = NaN
    everywhere), and the float64 oracle within 2 float32 ulps of it."""
    from oracle.gen_golden_normalize import STRIDE, clip_set, sha

    z = _norm_golden()
    for name, x in clip_set().items():
        y = of.normalize_f32(x)
        assert y.dtype == np.float32
        if f"norm_{name}_sha" in z:
            assert np.array_equal(y[::STRIDE], z[f"norm_{name}_sample"]), name
            assert sha(y) == str(z[f"norm_{name}_sha"]), name
        else:
            ref = z[f"norm_{name}"]
            assert np.array_equal(y, ref, equal_nan=True), name
        if name != "const":
            assert np.abs(of.normalize(x) - y).max() <= 2 * np.spacing(np.float32(1)), name
    assert np.isnan(z["norm_const"]).all()


def test_oracle_normalize_load_samples_windows():
    """load_samples(normalize=True) windows (zero-padded short tracks are
    normalised after padding): rebuilt from the fixture's window layout and
    normalised by of.normalize_f32, bit for bit."""
    from oracle.gen_golden_normalize import N, SR, STRIDE, hash_audio, sha

    z = _norm_golden()
    recs = {}
    for r, (k, ti, first, src, cnt) in enumerate(z["ls_rows"]):
        rec = recs.setdefault(int(k), hash_audio(SR * 20, 100 + int(k), 0.8))
        win = np.zeros(N, np.float32)
        win[first:first + cnt] = rec[src:src + cnt]
        y = of.normalize_f32(win)
        assert np.array_equal(y[::STRIDE], z["ls_sample"][r]), r
        assert sha(y) == str(z["ls_sha"][r]), r
    assert (z["ls_rows"][:, 4] < N).any()  # some windows are padded
