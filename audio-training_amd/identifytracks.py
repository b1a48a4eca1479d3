"""Track (signal) detection of the streaming predict path (reference
identifytracks.py:21-236, used by predict.py:736-740).

Host-side, as in the reference (a one-off pass per recording, not the batched
hot path): |STFT| (librosa.stft defaults: centred, constant padding, periodic
Hann) of the whole recording; a cell is "signal" when it exceeds twice its
frame's median and three times its frequency row's median; the binary map is
opened with a 4x4 box, dilated by (100 Hz of bins) x (0.25 s of frames) and
eroded by (a tenth of that height) x (the same width) -- the OpenCV
morphology (anchor at the box centre, borders ignored) restated with
scipy.ndimage min / max filters --; 8-connected components give time /
frequency boxes, which are filtered by size, then merged into tracks
(merge_signals, get_tracks_from_signals) with the reference's thresholds.

cv2 / librosa are not in the image: the morphology and the STFT are restated
from their published definitions (parity unpinned beyond that; the tests pin
the component boxes on synthetic recordings with known chirps).
"""
from __future__ import annotations

import math

import numpy as np

MAX_FRQUENCY = 48000 / 2
SIGNAL_WIDTH = 0.25
TOP_FREQ = 48000 / 2


def get_nfft(sr):
    """identifytracks.get_nfft (:13-18): a power of two near sr / 10."""
    return int(math.pow(2, round(math.log2(sr // 10))))


def stft_magnitude(frames, n_fft, hop_length, block=4096):
    """|librosa.stft(frames, n_fft, hop_length)| (centre=True, constant
    padding, periodic Hann) -> float32 [1 + n_fft // 2, 1 + len // hop]."""
    x = np.pad(np.asarray(frames, np.float32), (n_fft // 2, n_fft // 2))
    t = 1 + (len(x) - n_fft) // hop_length
    win = (0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n_fft) / n_fft)).astype(np.float32)
    out = np.empty((n_fft // 2 + 1, t), np.float32)
    base = np.arange(n_fft)
    for a in range(0, t, block):
        idx = np.arange(a, min(t, a + block))[:, None] * hop_length + base[None, :]
        out[:, a:a + idx.shape[0]] = np.abs(np.fft.rfft(x[idx] * win, axis=-1)).T
    return out


def mel_freq(f):
    """HTK mel (identifytracks.py:154-155)."""
    return 2595.0 * np.log10(1.0 + f / 700.0)


def segment_overlap(a, b):
    """Signed overlap length of two intervals (identifytracks.py:146-151)."""
    return (a[1] - a[0]) + (b[1] - b[0]) - (max(a[1], b[1]) - min(a[0], b[0]))


class Signal:
    """A time / frequency box (identifytracks.py:376-502)."""

    _next_id = 0

    def __init__(self, start, end, freq_start, freq_end, mass):
        self.id = Signal._next_id
        Signal._next_id += 1
        self.start, self.end = start, end
        self.freq_start, self.freq_end = freq_start, freq_end
        self.mass = mass
        self.mel_freq_start, self.mel_freq_end = mel_freq(freq_start), mel_freq(freq_end)
        self.predictions = []
        self.track_id = None

    def copy(self):
        return Signal(self.start, self.end, self.freq_start, self.freq_end, self.mass)

    @property
    def length(self):
        return self.end - self.start

    @property
    def mel_freq_range(self):
        return self.mel_freq_end - self.mel_freq_start

    @property
    def freq_range(self):
        return self.freq_end - self.freq_start

    def time_overlap(self, o):
        return segment_overlap((self.start, self.end), (o.start, o.end))

    def mel_freq_overlap(self, o):
        return segment_overlap((self.mel_freq_start, self.mel_freq_end), (o.mel_freq_start, o.mel_freq_end))

    def freq_overlap(self, o):
        return segment_overlap((self.freq_start, self.freq_end), (o.freq_start, o.freq_end))

    def enlarge(self, scale, min_track_length, max_extra=1):
        """Grow in time by `scale` (at least to min_track_length, at most
        max_extra s) and in frequency by `scale` (identifytracks.py:459-478)."""
        new_len = max(self.length * scale, min_track_length)
        ext = min(max_extra, new_len - self.length) / 2
        self.start = max(self.start - ext, 0)
        self.end = self.end + ext
        fr = self.freq_end - self.freq_start
        fext = (fr * scale - fr) / 2
        self.freq_end = int(self.freq_end + fext)
        self.freq_start = int(max(self.freq_start - fext, 0))
        self.mel_freq_start, self.mel_freq_end = mel_freq(self.freq_start), mel_freq(self.freq_end)

    def merge(self, o):
        self.start, self.end = min(self.start, o.start), max(self.end, o.end)
        self.freq_start, self.freq_end = min(self.freq_start, o.freq_start), max(self.freq_end, o.freq_end)
        self.mel_freq_start, self.mel_freq_end = mel_freq(self.freq_start), mel_freq(self.freq_end)
        self.mass += o.mass

    def to_array(self, decimals=1):
        a = [self.start, self.end, self.freq_start, self.freq_end]
        return list(np.round(np.array(a), decimals)) if decimals is not None else a

    def get_meta(self):
        meta = {"id": self.id, "start": self.start, "end": self.end, "freq_start": self.freq_start,
                "freq_end": self.freq_end,
                "positions": [{"y": self.freq_start / TOP_FREQ, "height": (self.freq_end - self.freq_start) / TOP_FREQ}],
                "predictions": [r.get_meta() for r in self.predictions]}
        if self.track_id is not None:
            meta["track_id"] = self.track_id
        return meta

    def __str__(self):
        return f"Signal: {self.start}-{self.end} f: {self.freq_start}-{self.freq_end} mass {self.mass}"


def get_end(frames, sr, mel=None):
    """Seconds of real data (identifytracks.py:21-48): the start of the first
    sr // hop frame chunk of the (120-band, break 1750 Hz, power 1) mel image
    whose max equals its min -- a digitally silent tail.  `mel` [M, T] may be
    passed in (the GPU front end computes it); else it is computed here."""
    hop = 281
    if mel is None:
        from acfe.frontend import mel_filterbank

        n_fft = get_nfft(sr)
        w = mel_filterbank(sr, 120, 50, 11000, n_fft, 1750)
        mel = w.astype(np.float32) @ stft_magnitude(frames, n_fft, hop)
    chunk = sr // hop
    start, end = 0, chunk
    while end < mel.shape[1]:
        d = mel[:, start:end]
        if np.amax(d) == np.amin(d):
            return start * hop // sr
        start, end = end, end + chunk
    return len(frames) / sr


def _box(h, w):
    # OpenCV replaces an empty structuring element by a 3x3 box
    return (3, 3) if h <= 0 or w <= 0 else (h, w)


def _box_max(a, h, w):
    """cv2.dilate with an h x w box (anchor at the centre, border ignored)."""
    from scipy.ndimage import maximum_filter

    return maximum_filter(a, size=_box(h, w), mode="constant", cval=0)


def _box_min(a, h, w):
    """cv2.erode with an h x w box (anchor at the centre, border ignored)."""
    from scipy.ndimage import minimum_filter

    return minimum_filter(a, size=_box(h, w), mode="constant", cval=1)


def signal_noise(frames, sr, hop_length=281, n_fft=1024, min_width=None, min_height=None, spectogram=None):
    """identifytracks.signal_noise (:51-143) -> (signals, |STFT|).  The
    reference overrides n_fft with 2048 (:55); so does this."""
    from scipy.ndimage import label

    n_fft = 2048
    if spectogram is None:
        spectogram = stft_magnitude(frames, n_fft, hop_length)
    freqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
    height = 0
    for i, f in enumerate(freqs):  # first bin above 100 Hz (+1)
        if f > 100:
            height = i + 1
            break
    spec = spectogram / np.amax(spectogram)
    row_med = np.median(spec, axis=1)[:, None]
    col_med = np.median(spec, axis=0)[None, :]
    signal = ((spec > 2 * col_med) & (spec > 3 * row_med)).astype(np.uint8)
    signal = _box_max(_box_min(signal, 4, 4), 4, 4)  # MORPH_OPEN, 4x4
    width = int(SIGNAL_WIDTH * sr / hop_length)
    signal = _box_max(signal, height, width)
    signal = _box_min(signal, height // 10, width)
    lab, n = label(signal, structure=np.ones((3, 3), np.uint8))  # 8-connectivity
    stats = []
    if n:
        from scipy.ndimage import find_objects

        area = np.bincount(lab.ravel(), minlength=n + 1)
        for k, sl in enumerate(find_objects(lab), start=1):
            top, left = sl[0].start, sl[1].start
            stats.append((left, top, sl[1].stop - left, sl[0].stop - top, int(area[k])))
    stats.sort(key=lambda s: s[0])
    if min_height is None:
        min_height = height - height // 10
    if min_width is None:
        min_width = 0.65 * width
    signals = []
    for s in stats:
        if not (s[2] > min_width and s[3] > min_height):
            continue
        max_freq = min(len(freqs) - 1, s[1] + s[3])
        signals.append(Signal(s[0] * 281 / sr, (s[0] + s[2]) * 281 / sr, freqs[s[1]], freqs[max_freq], s[4]))
    return signals, spectogram


def merge_signals(signals):
    """One merging pass (identifytracks.py:161-231) -> (signals, merged_any)."""
    to_delete = []
    something = False
    overlap_seconds = 1.5
    signals = sorted(signals, key=lambda s: s.mel_freq_end, reverse=True)
    signals = sorted(signals, key=lambda s: s.start)
    for s in signals:
        if s in to_delete:
            continue
        merged = False
        u = None
        for u in signals:
            if u in to_delete or u is s:
                continue
            same_side = (u.mel_freq_end < 1500 and s.mel_freq_end < 1500) or (u.mel_freq_end > 1500 and
                                                                            s.mel_freq_end > 1500)
            if not same_side:
                continue
            overlap = s.time_overlap(u)
            high = s.mel_freq_start > 1000 and u.mel_freq_start > 1000
            freq_overlap_time = 0.5 if high else 0.75
            time_diff = s.start - u.end if s.start > u.end else u.start - s.end
            mel_overlap = s.mel_freq_overlap(u)
            if (overlap > u.length * 0.75 and mel_overlap > -20) or overlap > overlap_seconds:
                s.merge(u)
                merged = True
                break
            if overlap > 0 and mel_overlap > u.mel_freq_range * freq_overlap_time:
                s.merge(u)
                merged = True
                break
            if mel_overlap > u.mel_freq_range * freq_overlap_time and time_diff <= 2:
                if u.mel_freq_end > s.mel_freq_range:
                    range_overlap = s.mel_freq_range / u.mel_freq_range
                else:
                    range_overlap = u.mel_freq_range / s.mel_freq_range
                if range_overlap < 0.75:
                    continue
                s.merge(u)
                merged = True
                break
        if merged:
            something = True
            to_delete.append(u)
    for s in to_delete:
        signals.remove(s)
    return signals, something


def get_tracks_from_signals(signals, end):
    """identifytracks.get_tracks_from_signals (:236-300): merge until stable,
    drop short boxes, enlarge, merge overlapping ones, drop narrow-band ones,
    split tracks longer than 6 s."""
    max_length = 6
    min_mel_range = 50
    merged = True
    while merged:
        signals, merged = merge_signals(signals)
    to_delete = []
    min_length_base, min_track_length, overlap_seconds = 0.35, 0.7, 1.5
    for s in signals:
        if s in to_delete:
            continue
        if s.length < min_length_base:
            to_delete.append(s)
            continue
        s.enlarge(1.4, min_track_length=min_track_length)
        s.end = min(end, s.end)
        for s2 in signals:
            if s2 in to_delete or s2 is s:
                continue
            overlap = s.time_overlap(s2)
            if overlap > 0.7 * min(s.length, s2.length) or overlap > overlap_seconds:
                s.merge(s2)
                to_delete.append(s2)
    for s in to_delete:
        signals.remove(s)
    signals = [s for s in signals if s.mel_freq_range >= min_mel_range]
    final = []
    for s in signals:
        if s.length > max_length:
            splits = math.ceil(s.length / max_length)
            length = s.length / splits
            start = s.start
            for _ in range(splits):
                ns = s.copy()
                ns.start, ns.end = start, start + length
                final.append(ns)
                start = ns.end
        else:
            final.append(s)
    return final
