"""build.py -> audiomodel.py -> predict.py, the reference's three entry points
(build.py:679, audiomodel.py:1985, predict.py:726) on the acfe path."""
import json
import sys

import numpy as np
import pytest
import torch

from conftest import PKG


def _build(tmp_path, n=24, spectrogram=True):
    import build

    extra = [] if spectrogram else ["--no-spectrogram"]
    assert build.main([str(tmp_path / "ds"), "--synthetic", str(n), "--labels", "bird,noise", "--shards", "2"]
                      + extra) == 0
    return tmp_path / "ds" / "training-data"


def test_build_synthetic_records(tmp_path):
    import tfrecord as tfr

    td = _build(tmp_path)
    meta = json.loads((td / "training-meta.json").read_text())
    assert meta["labels"] == ["bird", "noise"] and meta["type"] == "audio"
    total = 0
    seen = {}
    for split in ("train", "validation", "test"):
        files = sorted((td / split).glob("*.tfrecord"))
        n = 0
        for f in files:
            for rec in tfr.read_records(f):
                ex = tfr.parse_audio_example(rec)
                assert ex["raw"].shape == (144000,) and ex["text"] in ("bird", "noise")
                sp = tfr.parse_audio_example(rec, load_raw=False)["spectrogram"]
                assert sp.shape == (2049, 513) and sp.dtype == np.float32
                seen.setdefault(ex["rec_id"], set()).add(split)
                n += 1
        assert n == sum(meta["counts"][split]["sample_counts"].values())
        total += n
    assert total == 24
    assert all(len(v) == 1 for v in seen.values())  # no recording in two splits


def test_stored_spectrogram_matches_oracle():
    """build.stft_magnitude = the audio/spectogram audiodataset.load_data stores
    (:1302-1303: |librosa.stft(normalize_data(clip))|, center=True, constant
    padding) against the float64 oracle restatement (oracle.frontend.stft_center)."""
    import build
    from oracle import frontend as of

    clip = build.synth_clip(np.random.default_rng(5), False)
    got = build.stft_magnitude(clip)
    ref = np.abs(of.stft_center(of.normalize(clip)[None], 4096, 281, "constant"))[0]
    assert got.shape == ref.shape == (2049, 513)
    assert np.abs(got - ref).max() <= 2e-6 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("load_raw", [False, True], ids=["spectrogram", "raw"])
def test_train_checkpoint_predict(tmp_path, cuda, load_raw):
    """The default CLI path trains on the stored spectrograms (--load-raw is a
    count flag defaulting to off, audiomodel.py:2344-2349); --load-raw trains on
    the raw audio with the GPU STFT and mix_up."""
    import audiomodel
    import predict
    from scipy.io import wavfile

    td = _build(tmp_path, 16)
    args = audiomodel.parse_args(["run1", "-d", str(td), "--epochs", "1", "--batch-size", "4", "--model-name",
                                  "wr-resnet-bird", "--n_mels", "128", "--checkpoint-dir", str(tmp_path / "ck")]
                                 + (["--load-raw"] if load_raw else []))
    hist = audiomodel.train_model(args)
    assert np.isfinite(hist["loss"][0])
    ck = tmp_path / "ck" / "run1"
    meta = json.loads((ck / "metadata.txt").read_text())
    assert (ck / "model.pt").exists() and meta["labels"] == ["bird", "noise"]
    assert (ck / "model.weights.h5").exists()  # Keras 3 layout, as the reference's checkpoints
    assert meta["power"] == (2 if load_raw else 1) and meta["load_raw"] == load_raw
    # 10 s synthetic recording -> 8 windows at 1 s stride
    import build

    rng = np.random.default_rng(3)
    rec = np.concatenate([build.synth_clip(rng, False) for _ in range(3)] + [build.synth_clip(rng, True)[:48000]])
    wavfile.write(tmp_path / "rec.wav", 48000, (rec * 32767).astype(np.int16))
    p = predict.Predictor(ck)
    r = p.predict_file(tmp_path / "rec.wav", stride=1.0, batch_size=4)
    assert r["windows"] == 8
    assert set(r["mean"]) == {"bird", "noise"} and all(0 <= v <= 1 for v in r["mean"].values()), (r, hist)
    # track mode gathers windows on the host: the same windows read in place
    # by the fused front end give the same probabilities
    wins = np.stack([rec[k * 48000:(k + 3) * 48000] for k in range(8)])
    a, b = p.predict_clips(wins, batch_size=8), p.predict_windows(rec, 1.0, batch_size=8)
    assert np.abs(a - b).max() < 2e-3
    tracks, end = p.predict_tracks(rec, batch_size=4, rng=np.random.RandomState(0))
    assert end == pytest.approx(len(rec) / 48000)
    for t in tracks:
        (res,) = t.predictions
        assert res.labels or res.raw_tag in ("bird", "noise")
    predict.main([str(ck), "--file", str(tmp_path / "rec.wav"), "--mode", "tracks"])
    # the same checkpoint read through its Keras weights file (no model.pt):
    # identical model outputs (PCEN at its default init on both sides is not
    # compared: the reference's wr-resnet models carry no PCEN)
    import shutil

    kd = tmp_path / "keras_ck"
    kd.mkdir()
    shutil.copy(ck / "metadata.txt", kd / "metadata.txt")
    shutil.copy(ck / "model.weights.h5", kd / "model.weights.h5")
    pk = predict.Predictor(kd)
    for (n1, t1), (n2, t2) in zip(p.model.state_dict().items(), pk.model.state_dict().items()):
        assert n1 == n2 and torch.equal(t1.cpu(), t2.cpu()), n1


@pytest.mark.gpu
def test_config_p_plumbing(tmp_path, cuda):
    """BASELINE config P (build.py:679-814 -> audiomodel.py:405-567): a 256-clip
    synthetic 2-class (bird / noise) TFRecord set, wr_resnet (the
    `--model-name wr-resnet` model), batch 8, 128 mels with raw records, one
    epoch through the TFRecord loader on the GPU path; clips/s reported."""
    import time

    import audiomodel

    t0 = time.perf_counter()
    td = _build(tmp_path, 256, spectrogram=False)
    t_build = time.perf_counter() - t0
    meta = json.loads((td / "training-meta.json").read_text())
    n_train = sum(meta["counts"]["train"]["sample_counts"].values())
    args = audiomodel.parse_args(["p", "-d", str(td), "--epochs", "1", "--batch-size", "8", "--model-name",
                                  "wr-resnet", "--n_mels", "128", "--load-raw", "--checkpoint-dir",
                                  str(tmp_path / "ck")])
    hist = audiomodel.train_model(args)
    assert np.isfinite(hist["loss"][0]) and np.isfinite(hist["val_loss"][0])
    assert 0.0 <= hist["val_accuracy"][0] <= 1.0
    print(f"config P: build {t_build:.1f} s for 256 clips, {n_train} train clips, "
          f"{hist['clips_per_s'][0]:.1f} clips/s (loader + GPU step, batch 8)")
