"""Generate golden fixtures for the streaming path's index work from the
REFERENCE identifytracks.py and predict_utils.py.

Test infrastructure only (see oracle/__init__.py).  Run in the build container,
where /root/reference exists; the .npz output is committed under tests/golden/
and is the only thing that travels.  Both reference modules import heavy
libraries at module top that are absent here (librosa, cv2, plot_utils,
tensorflow); the functions pinned below never call them, so the imports are
satisfied by empty stub modules (librosa gets `fft_frequencies`, as in
oracle/gen_golden.py, for custommel).  Pinned reference functions:

  * identifytracks.merge_signals (:162-233), get_tracks_from_signals (:236-301),
    Signal (:376-484: enlarge / merge / overlaps) -- seeded synthetic signal
    lists shaped like signal_noise's output (frame-quantised times, FFT-bin
    frequencies), with and without splits of long tracks;
  * identifytracks.get_end (:21-48) -- the chunk scan, with librosa.stft
    stubbed to return a given |S| and the reference custommel.mel_spec real;
  * predict_utils.load_samples (:9-150) -- the window cutting (short-track
    centring, edges, stride, pad_short_tracks, random pad offsets from a
    seeded np.random), with get_spect stubbed to return the cut window and
    normalize=False, so each window is recorded as (pad_left, src_start, n_src)
    over a ramp recording whose sample i holds i + 1.

Not pinnable here: identifytracks.signal_noise (cv2 morphology and connected
components) and the STFTs (librosa) -- restated, parity unpinned.

Usage: python oracle/gen_golden_tracks.py [--ref /root/reference] [--out tests/golden]
"""
import argparse
import sys
import types
from pathlib import Path

import numpy as np

SR = 48000


def _stubs():
    lib = types.ModuleType("librosa")
    lib.fft_frequencies = lambda *, sr=22050, n_fft=2048: np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    lib._stft_result = None

    def stft(*a, **k):
        return lib._stft_result

    lib.stft = stft
    sys.modules["librosa"] = lib
    for name in ("cv2", "plot_utils", "tensorflow"):
        sys.modules[name] = types.ModuleType(name)
    return lib


def _signal_lists(rng, n_cases):
    """Signal boxes shaped like signal_noise's (identifytracks.py:136-141):
    start / end on the 281-sample frame grid, frequencies on the 2048-point
    FFT bin grid, integer masses; clustered so that every merge rule fires."""
    cases = []
    for c in range(n_cases):
        dur = float(rng.choice([12.0, 30.0, 60.0]))
        n = int(rng.integers(2, 28))
        centres = rng.uniform(0, dur, int(rng.integers(1, 5)))
        bands = rng.choice([200.0, 900.0, 1800.0, 3000.0, 5000.0, 9000.0], size=len(centres))
        boxes = []
        for _ in range(n):
            k = int(rng.integers(0, len(centres)))
            t0 = max(0.0, centres[k] + rng.normal(0, 1.5))
            ln = float(rng.choice([rng.uniform(0.1, 0.5), rng.uniform(0.3, 3.0), rng.uniform(4.0, 15.0)],
                                  p=[0.25, 0.6, 0.15]))
            f0 = max(0.0, bands[k] * rng.uniform(0.6, 1.4))
            fw = bands[k] * rng.uniform(0.05, 1.2)
            fr0, fr1 = t0 * SR / 281, (t0 + ln) * SR / 281
            b0, b1 = int(f0 * 2048 / SR), int((f0 + fw) * 2048 / SR) + 1
            boxes.append((int(fr0) * 281 / SR, int(fr1) * 281 / SR, b0 * SR / 2048, min(b1, 1024) * SR / 2048,
                          int(rng.integers(20, 5000))))
        end = dur if c % 3 else dur * 0.7  # some recordings end before their last box
        cases.append((boxes, end))
    return cases


# get_end cases: (seconds, silent from (s) or None)
GET_END_CASES = [(10, None), (10, 6.3), (7, 2.0), (5, 0.0), (20, 17.5), (9, 8.9)]


def get_end_spectrogram(k, n, silent_from):
    """The |S| librosa.stft is stubbed to return for get_end case k (also
    rebuilt by tests/test_identifytracks.py): PCG64-seeded noise, constant
    (max == min over a chunk) from `silent_from` seconds on."""
    T = 1 + n // 281
    S = np.random.default_rng(1000 + k).random((4096 // 2 + 1, T), dtype=np.float32) + np.float32(0.01)
    if silent_from is not None:
        S[:, int(silent_from * SR / 281):] = 0.0
    return S


def _tracks(it, boxes):
    return [it.Signal(*b) for b in boxes]


def _pack(sigs):
    return np.array([(s.start, s.end, s.freq_start, s.freq_end, s.mass) for s in sigs], np.float64).reshape(-1, 5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parent.parent / "tests" / "golden"))
    a = ap.parse_args()
    lib = _stubs()
    sys.path.insert(0, a.ref)
    import custommel
    import identifytracks as it
    import predict_utils as pu

    out = {}
    rng = np.random.default_rng(20260417)

    # --- merge_signals (one pass) and get_tracks_from_signals ------------------
    cases = _signal_lists(rng, 60)
    offs, ins, ends, one, one_off, tr, tr_off, merged_flags = [0], [], [], [], [0], [], [0], []
    for boxes, end in cases:
        ins.append(np.array(boxes, np.float64))
        offs.append(offs[-1] + len(boxes))
        ends.append(end)
        sigs, m = it.merge_signals(_tracks(it, boxes))
        merged_flags.append(int(m))
        one.append(_pack(sigs))
        one_off.append(one_off[-1] + len(sigs))
        t = it.get_tracks_from_signals(_tracks(it, boxes), end)
        tr.append(_pack(t))
        tr_off.append(tr_off[-1] + len(t))
    out.update(sig_in=np.concatenate(ins), sig_off=np.array(offs, np.int64), sig_end=np.array(ends, np.float64),
               merge_out=np.concatenate(one), merge_off=np.array(one_off, np.int64),
               merge_flag=np.array(merged_flags, np.int64), tracks_out=np.concatenate(tr),
               tracks_off=np.array(tr_off, np.int64))
    print("signal cases", len(cases), "boxes", offs[-1], "one-pass", one_off[-1], "tracks", tr_off[-1])

    # --- get_end: the chunk scan over the reference mel_spec of a given |S| ----
    ge_len, ge_end, ge_sum = [], [], []
    for k, (secs, silent_from) in enumerate(GET_END_CASES):
        n = SR * secs
        lib._stft_result = get_end_spectrogram(k, n, silent_from)
        ge_len.append(n)
        ge_end.append(float(it.get_end(np.zeros(n, np.float32), SR)))
        ge_sum.append(float(custommel.mel_spec(lib._stft_result, SR, 4096, 281, 120, 50, 11000, 1750, power=1).sum()))
    out.update(getend_len=np.array(ge_len, np.int64), getend_end=np.array(ge_end, np.float64),
               getend_melsum=np.array(ge_sum, np.float64))
    print("get_end", ge_end)

    # --- load_samples window cutting -----------------------------------------
    pu.get_spect = lambda data, *args, **kw: np.array(data, copy=True)
    win_rows, win_case = [], []
    case_meta = []
    for k, (secs, boxes, pad, seed, stride) in enumerate([
        (20, [(5.0, 6.2), (2.0, 7.5), (0.2, 1.0), (19.3, 19.9), (18.0, 20.0), (0.0, 3.0), (4.0, 4.05)], False, 0, 1),
        (20, [(5.0, 6.2), (2.0, 7.5), (0.2, 1.0), (19.3, 19.9), (18.0, 20.0), (0.0, 3.0), (4.0, 4.05)], True, 1, 1),
        (12, [(1.0, 5.5), (4.0, 5.0), (10.9, 12.0), (0.0, 12.0)], False, 2, 1),
        (12, [(1.0, 5.5), (4.0, 5.0), (10.9, 12.0), (0.0, 12.0)], True, 3, 1),
        (2, [(0.1, 0.5), (0.0, 2.0)], False, 4, 1),  # recording shorter than a window
        (2, [(0.1, 0.5), (0.0, 2.0)], True, 5, 1),
        (30, [(3.3, 9.71), (12.0, 12.4), (25.0, 29.99)], False, 6, 1),
        (30, [(3.3, 9.71), (12.0, 12.4), (25.0, 29.99)], False, 7, 2),
    ]):
        n = SR * secs
        frames = np.arange(1, n + 1, dtype=np.float32)  # sample i holds i + 1 (exact in f32)
        tracks = [it.Signal(s, e, 1000.0, 3000.0, 1) for s, e in boxes]
        tracks.append(it.Signal(1.0, 2.0, 12000.0, 15000.0, 1))  # above fmax: not classified
        np.random.seed(seed)
        res = pu.load_samples(frames, SR, tracks, stride=stride, normalize=False, pad_short_tracks=pad)
        for ti, wins in enumerate(res):
            for w in wins:
                w = np.asarray(w)
                assert w.shape == (SR * 3,)
                nz = np.flatnonzero(w)
                first = int(nz[0]) if len(nz) else 0
                cnt = len(nz)
                src = int(w[first]) - 1 if cnt else 0
                assert np.array_equal(w[first:first + cnt], np.arange(src + 1, src + cnt + 1, dtype=np.float32))
                assert not w[:first].any() and not w[first + cnt:].any()
                win_rows.append((ti, first, src, cnt))
                win_case.append(k)
        case_meta.append((secs, int(pad), seed, stride, len(tracks)))
        out[f"ls_tracks{k}"] = np.array([(t.start, t.end, t.freq_start, t.freq_end) for t in tracks], np.float64)
    out.update(ls_meta=np.array(case_meta, np.int64), ls_rows=np.array(win_rows, np.int64),
               ls_case=np.array(win_case, np.int64))
    print("load_samples windows", len(win_rows))

    dst = Path(a.out) / "tracks_golden.npz"
    np.savez_compressed(dst, **out)
    print("wrote", dst)


if __name__ == "__main__":
    main()
