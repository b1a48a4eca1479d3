"""Track detection of the predict path (audio-training_amd/identifytracks.py,
restating reference identifytracks.py:21-300 and predict_utils.load_samples).

cv2 and librosa are absent, so the morphology is pinned against a direct
restatement of OpenCV's published erode / dilate definition (anchor at the
box centre, out-of-image pixels ignored), and the detector against synthetic
recordings with chirps at known times and frequencies."""
import numpy as np
import pytest

import identifytracks as it
import predict

SR = 48000


def _cv_morph(a, h, w, op):
    """dst(y, x) = op over the h x w box at anchor (h // 2, w // 2) of the
    in-image src pixels (cv::dilate / cv::erode with the default border)."""
    H, W = a.shape
    out = np.empty_like(a)
    for y in range(H):
        for x in range(W):
            y0, x0 = max(0, y - h // 2), max(0, x - w // 2)
            y1, x1 = min(H, y - h // 2 + h), min(W, x - w // 2 + w)
            out[y, x] = op(a[y0:y1, x0:x1])
    return out


@pytest.mark.parametrize("h,w", [(4, 4), (6, 9), (3, 5), (1, 7)])
def test_morphology_matches_opencv_definition(h, w):
    rng = np.random.default_rng(h * 10 + w)
    a = (rng.random((23, 31)) < 0.3).astype(np.uint8)
    assert np.array_equal(it._box_max(a, h, w), _cv_morph(a, h, w, np.max))
    assert np.array_equal(it._box_min(a, h, w), _cv_morph(a, h, w, np.min))
    # an empty structuring element is OpenCV's 3x3 default
    assert np.array_equal(it._box_min(a, 0, w), _cv_morph(a, 3, 3, np.min))


def test_stft_magnitude_matches_direct_dft():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(3000).astype(np.float32)
    got = it.stft_magnitude(x, 256, 97)
    xp = np.pad(x.astype(np.float64), 128)
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(256) / 256)
    t = 1 + (len(xp) - 256) // 97
    ref = np.abs(np.stack([np.fft.rfft(xp[i * 97:i * 97 + 256] * win) for i in range(t)], 1))
    assert got.shape == ref.shape == (129, 1 + 3000 // 97)
    assert np.abs(got - ref).max() <= 1e-4 * ref.max()


def _recording(chirps, seconds=20, noise=0.003, seed=0):
    rng = np.random.default_rng(seed)
    n = SR * seconds
    x = rng.normal(0, noise, n)
    t = np.arange(n) / SR
    for on, dur, f0, f1 in chirps:
        m = (t >= on) & (t < on + dur)
        tt = t[m] - on
        x[m] += 0.3 * np.sin(2 * np.pi * (f0 * tt + 0.5 * (f1 - f0) / dur * tt * tt))
    return x.astype(np.float32)


CHIRPS = [(2.0, 1.0, 3000, 4000), (8.0, 0.6, 6000, 5000), (14.0, 2.5, 1500, 2500)]


def test_signals_and_tracks_on_synthetic_chirps():
    x = _recording(CHIRPS)
    signals, spec = it.signal_noise(x, SR)
    assert spec.shape == (1025, 1 + len(x) // 281)
    # every chirp is covered by a detected box, and every box lies on a chirp
    for on, dur, f0, f1 in CHIRPS:
        assert any(s.start <= on + 0.05 and s.end >= on + dur - 0.05 and s.freq_start <= min(f0, f1)
                   and s.freq_end >= max(f0, f1) for s in signals), (on, [str(s) for s in signals])
    for s in signals:
        assert any(s.start < on + dur + 0.3 and s.end > on - 0.3 for on, dur, _, _ in CHIRPS), str(s)
    tracks = it.get_tracks_from_signals(signals, 20.0)
    assert len(tracks) == 3
    tracks.sort(key=lambda s: s.start)
    for t, (on, dur, f0, f1) in zip(tracks, CHIRPS):
        assert t.start <= on and t.end >= on + dur and t.end - t.start <= max(dur * 1.4, 0.7) + 1.1
        assert t.freq_start <= min(f0, f1) and t.freq_end >= max(f0, f1)
        assert t.mel_freq_range >= 50


def test_long_tracks_are_split():
    x = _recording([(1.0, 13.0, 2000, 3000)])
    tracks = it.get_tracks_from_signals(it.signal_noise(x, SR)[0], 20.0)
    assert len(tracks) == 3  # 13 s (+ enlargement) > 2 * 6 s -> 3 equal pieces
    lens = [t.length for t in tracks]
    assert max(lens) - min(lens) < 1e-9 and max(lens) <= 6
    for a, b in zip(tracks, tracks[1:]):
        assert abs(a.end - b.start) < 1e-9


def test_merge_rules():
    a = it.Signal(1.0, 2.0, 2000, 4000, 10)
    b = it.Signal(1.2, 1.9, 2500, 3800, 5)  # inside a in time, overlapping in mel
    c = it.Signal(10.0, 10.5, 2000, 4000, 7)  # far away
    out, merged = it.merge_signals([a, b, c])
    assert merged and len(out) == 2
    m = [s for s in out if s.start < 5][0]
    assert (m.start, m.end, m.freq_start, m.freq_end, m.mass) == (1.0, 2.0, 2000, 4000, 15)
    # opposite sides of the 1500-mel line never merge
    lo, hi = it.Signal(1.0, 2.0, 100, 900, 1), it.Signal(1.0, 2.0, 3000, 6000, 1)
    out, merged = it.merge_signals([lo, hi])
    assert not merged and len(out) == 2


def test_get_end_finds_silent_tail():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.normal(0, 0.1, SR * 10), np.zeros(SR * 10)]).astype(np.float32)
    assert it.get_end(x, SR) == 10
    assert it.get_end(rng.normal(0, 0.1, SR * 5).astype(np.float32), SR) == 5.0


def test_track_windows_follow_load_samples():
    rng = np.random.default_rng(2)
    frames = rng.standard_normal(SR * 20).astype(np.float32)
    short = it.Signal(5.0, 6.2, 1000, 3000, 1)  # centred in one 3 s window
    long_ = it.Signal(2.0, 7.5, 1000, 3000, 1)  # 5.5 s -> windows at +0, +1, +2 s
    edge = it.Signal(0.2, 1.0, 1000, 3000, 1)  # near the start: window from 0
    high = it.Signal(3.0, 4.0, 12000, 15000, 1)  # above fmax: not classified
    wins = predict.track_windows(frames, SR, [short, long_, edge, high], rng=np.random.RandomState(0))
    n = 3 * SR
    missing = n - (int(6.2 * SR) - 5 * SR)
    s0 = 5 * SR - missing // 2
    assert wins[0].shape == (1, n) and np.array_equal(wins[0][0], frames[s0:s0 + n])
    assert wins[1].shape == (3, n)
    for k in range(3):
        assert np.array_equal(wins[1][k], frames[(2 + k) * SR:(5 + k) * SR])
    assert np.array_equal(wins[2][0], frames[:n])
    assert wins[3].shape == (0, n)
    # a recording shorter than a window: zero padded at a random offset
    tiny = frames[:SR]
    w = predict.track_windows(tiny, SR, [it.Signal(0.1, 0.5, 1000, 3000, 1)], rng=np.random.RandomState(0))[0]
    nz = np.flatnonzero(w[0])
    assert w.shape == (1, n) and np.array_equal(w[0][nz[0]:nz[0] + SR], tiny)


def test_track_windows_pad_short_tracks():
    """pad_short_tracks=True (predict_utils.py:75-77): a short track is NOT
    re-centred; its own samples are zero padded at a random offset into one
    window, and a track longer than one window still gets one window per
    stride while end <= its length."""
    rng = np.random.default_rng(4)
    frames = rng.standard_normal(SR * 12).astype(np.float32)
    short = it.Signal(4.0, 5.0, 1000, 3000, 1)
    long_ = it.Signal(1.0, 5.5, 1000, 3000, 1)
    w = predict.track_windows(frames, SR, [short, long_], pad_short_tracks=True, rng=np.random.RandomState(1))
    n = 3 * SR
    assert w[0].shape == (1, n)
    nz = np.flatnonzero(w[0][0])
    assert np.array_equal(w[0][0][nz[0]:nz[0] + SR], frames[4 * SR:5 * SR])
    assert w[1].shape == (2, n)  # windows at +0 and +1 s; +2 s would end past 4.5 s
    for k in range(2):
        assert np.array_equal(w[1][k], frames[(1 + k) * SR:(4 + k) * SR])
